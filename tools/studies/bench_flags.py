"""Run bench.py with ops module flags flipped (in-process A/B of kernel paths
without environment knobs):

    python -m tools.studies.bench_flags GG_FUSE_RESOLVE=0 -- --model deepfm --qps 0

Every NAME=0/1 before ``--`` sets ``distributed_tf_serving_amd.ops.NAME``; the
rest is bench.py's command line.
"""
from __future__ import annotations

import os
import runpy
import sys


def main() -> None:
    argv = sys.argv[1:]
    split = argv.index("--") if "--" in argv else len(argv)
    flags, rest = argv[:split], argv[split + 1:]
    from distributed_tf_serving_amd import ops

    for f in flags:
        name, val = f.split("=", 1)
        if not hasattr(ops, name):
            raise SystemExit(f"ops has no flag {name}")
        setattr(ops, name, val not in ("0", "false", "False"))
        print(f"[bench_flags] ops.{name} = {getattr(ops, name)}", file=sys.stderr)
    bench = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "bench.py")
    sys.argv = [bench] + rest
    runpy.run_path(bench, run_name="__main__")


if __name__ == "__main__":
    main()
