"""tools/prof_summary.py on a synthetic trace database (the rocpd tables it reads)."""
import sqlite3

from tools.prof_summary import summarize


def test_step_timeline_gap_anatomy(tmp_path):
    db = str(tmp_path / "t.db")
    c = sqlite3.connect(db)
    c.execute("create table kernels(name text, start int, end int, duration int)")
    c.execute("create table memory_copies(name text, start int, end int, duration int, size int)")
    us = 1000
    # steps every 120 us: a 100 us kernel; each step's 5 MB copy lands 10 us after the previous kernel ends
    for k in range(6):
        t = k * 120 * us
        c.execute("insert into kernels values (?, ?, ?, ?)", ("gather_mlp_kernel", t, t + 100 * us, 100 * us))
        if k:
            c.execute("insert into memory_copies values (?, ?, ?, ?, ?)",
                      ("MEMORY_COPY_HOST_TO_DEVICE", t - 100 * us, t - 10 * us, 90 * us, 5 << 20))
    c.commit()
    out = summarize(db, step_kernel="gather_mlp", min_us=60)
    assert "period 120.0 us, kernels busy 100.0 us, GPU idle 20.0 us" in out
    assert "landed 10.0 us after the previous step's last kernel ended" in out
    assert "started 10.0 us after that copy landed" in out
