"""Candidate fan-out across the GPUs of a node (RCCL over xGMI).

The reference client splits one request's candidates across N TF-Serving hosts
and gathers the scores back (reference DCNClient.java:46-74 split, :146-164
dispatch + join). Here the hosts are the ranks of one process group and the
network hop becomes collectives on device buffers of packed rows
(:mod:`..serving.packing`):

``scatter``   the reference topology: rank 0 is the only front door; its
              ``world * B`` rows are scattered (C1) and per-rank scores are
              gathered back to it (C2).
``alltoall``  every rank is a front door; each rank's ``B`` rows are split
              across all GPUs and scores return to the submitting rank with a
              second all-to-all. Same per-request fan-out as ``scatter`` but
              the host->GPU traffic is spread over every GPU's PCIe link, so it
              scales with N instead of saturating rank 0's link.
``local``     no fan-out (each rank serves its own rows): the baseline.

``scatter`` on one node runs through rank 0's shared request arenas when the
engine gets a ``shared_scatter`` segment (parallel/shared_scatter.py,
csrc/runtime/shared_scatter.h): every rank DMAs only its share of rank 0's
batch over its own PCIe link, runs the LOCAL step on it and writes its scores
into rank 0's shared output - no collective in the step. The RCCL scatter is
the fallback.

Per step every rank runs, on its own HIP streams::

    H2D (copy stream) -> collective -> graph(forward) -> collective -> D2H

with two pipeline slots, so step k+1's H2D and host-side decode overlap step
k's compute. Equal split sizes keep every collective shape static (no count
exchange; graph-friendly).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from ..serving.executor import ShardExecutor
from .dist import DistContext

MODES = ("alltoall", "scatter", "local")


class StepTimeout(RuntimeError):
    """A step did not finish within the step timeout (a peer rank is gone, a
    communicator failed, or the device hangs): the caller fails the step's
    requests instead of blocking forever."""


class _RunnerEvent:
    """Adapter so a StepHandle can wait on a native StepRunner slot."""

    __slots__ = ("runner", "slot", "comms")

    def __init__(self, runner, slot, comms=()):
        self.runner, self.slot, self.comms = runner, slot, [c for c in comms if c is not None]

    def synchronize(self, timeout_s: Optional[float] = None):
        if timeout_s is None:
            self.runner.wait(self.slot)
            return
        ok, err = self.runner.wait_for(self.slot, float(timeout_s), self.comms)
        if not ok:
            raise StepTimeout(f"GPU step failed: {err}")

    def query(self) -> bool:
        return self.runner.query(self.slot)


class _ScatterEvent:
    """A shared-scatter step: this rank's step, then (rank 0) every rank's share."""

    __slots__ = ("eng", "slot", "k")

    def __init__(self, eng, slot, k):
        self.eng, self.slot, self.k = eng, slot, k

    def synchronize(self, timeout_s: Optional[float] = None):
        ok, err = self.eng.scatter.wait(self.eng.runner(), self.slot, self.k, float(timeout_s or 1e6))
        if not ok:
            raise StepTimeout(f"shared scatter step failed: {err}")

    def query(self) -> bool:  # polled by _wait_event: wait in full instead
        self.synchronize(self.eng.step_timeout_s)
        return True


def _wait_event(ev, timeout_s: Optional[float]) -> None:
    """Bounded wait on a torch event or a _RunnerEvent."""
    if isinstance(ev, (_RunnerEvent, _ScatterEvent)) or timeout_s is None:
        ev.synchronize(timeout_s) if isinstance(ev, (_RunnerEvent, _ScatterEvent)) else ev.synchronize()
        return
    deadline = time.monotonic() + timeout_s
    spins = 0
    while not ev.query():
        if time.monotonic() > deadline:
            raise StepTimeout(f"GPU step not finished after {timeout_s:.1f} s")
        spins += 1
        time.sleep(0 if spins < 200 else 5e-5)


@dataclass
class StepHandle:
    B: int
    slot: int
    host_out: torch.Tensor
    event: Optional[object] = None
    t_submit: float = 0.0
    t_done: float = 0.0
    timeout_s: Optional[float] = None

    def wait(self) -> torch.Tensor:
        """Scores of the step; raises StepTimeout past the engine's step timeout."""
        if self.event is not None:
            _wait_event(self.event, self.timeout_s)
        self.t_done = time.perf_counter()
        return self.host_out


class FanoutEngine:
    def __init__(self, executor: ShardExecutor, ctx: DistContext, mode: str = "alltoall", group=None,
                 step_graphs: bool = True, native_launch: bool = True, ingest: str = "packed", arena=None,
                 native_fanout: bool = True, force_fanout: bool = False, shared_scatter=None):
        """``ingest="packed"``: the host decodes into packed rows (host_in) and
        the H2D moves rows. ``ingest="arena"``: the host only parses request
        framing into a request arena (serving/arena.py); the H2D moves the raw
        request bytes and the GPU unpacks rows (csrc/kernels/ingest.hip).

        ``native_fanout`` (GPU, world > 1): the whole fan-out step is enqueued
        from C++ (StepRunner.launch_fanout) with native RCCL communicators
        (csrc/comm) - ingress and egress exchanges on their own streams and
        communicators, overlapping the forward graph. ``force_fanout`` keeps
        the fan-out mode on a 1-rank job (exercises that path on one GPU)."""
        if mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}")
        if ingest not in ("packed", "arena"):
            raise ValueError("ingest must be 'packed' or 'arena'")
        if ingest == "arena" and arena is None:
            raise ValueError("arena ingest needs an ArenaLayout")
        self.ingest = ingest
        self.arena = arena
        self._host_arena: Dict[int, torch.Tensor] = {}
        self._dev_arena: Dict[int, torch.Tensor] = {}
        self.ex = executor
        self.ctx = ctx
        self.world = ctx.world if ctx.is_distributed else 1
        self.rank = ctx.rank if ctx.is_distributed else 0
        self.mode = mode if (self.world > 1 or force_fanout) else "local"
        self.group = group
        self.native_fanout = native_fanout
        self.force_fanout = force_fanout
        # shared-arena scatter (scatter mode, one node): the step is local
        self.scatter = shared_scatter if (self.mode == "scatter" and ingest == "arena") else None
        self._local_arena: Dict[int, torch.Tensor] = {}
        self._cin = self._cout = None
        self._cprog = None  # step-program communicator (embedding-parallel models)
        self._programs: Dict[Tuple[int, int], object] = {}
        self._prog_bufs: Dict[Tuple[int, int], dict] = {}
        self.program_active = False
        self._program_buckets: set = set()  # buckets whose step is a two-lane program
        self._ingress_graph: Dict[Tuple[int, int], object] = {}
        self._split: Dict[Tuple[int, int], object] = {}  # two-lane fan-out forward (_capture_split)
        self._seqs: Dict[int, object] = {}
        self.native_fanout_active = False
        self.self_checks: list = []  # self_check() results: {bucket, rows, max_abs_diff}
        self._native_disabled = False
        self.layout = executor.layout
        self.dev = executor.device
        self.cuda = self.dev.type == "cuda"
        if self.cuda:
            self.h2d_stream = torch.cuda.Stream(self.dev)
            self.d2h_stream = torch.cuda.Stream(self.dev)
        self._host_in: Dict[Tuple[int, int], torch.Tensor] = {}
        self._host_out: Dict[Tuple[int, int], torch.Tensor] = {}
        self._dev_send: Dict[Tuple[int, int], torch.Tensor] = {}
        self._dev_back: Dict[Tuple[int, int], torch.Tensor] = {}
        self._ev_in_free: Dict[int, object] = {}
        self._ev_out_free: Dict[int, object] = {}
        self.step_graphs = step_graphs
        self.native_launch = native_launch
        self._runner = None
        self._step_graph: Dict[Tuple[int, int], object] = {}
        # bound on every StepHandle.wait (None = unbounded): a multi-rank step
        # waits on its peers, and a dead peer must not block this rank forever
        self.step_timeout_s: Optional[float] = float(os.environ.get("DTFS_STEP_TIMEOUT_S", "30"))

    # -- geometry ------------------------------------------------------------
    def contrib_rows(self, B: int) -> int:
        """Rows this rank submits per step when every GPU computes B rows."""
        if self.mode == "scatter":
            return self.world * B if self.rank == 0 else 0
        return B

    def check_bucket(self, B: int) -> None:
        if self.mode == "alltoall" and B % self.world:
            raise ValueError(f"bucket {B} must be divisible by world size {self.world} for all-to-all fan-out")

    def host_in(self, B: int, slot: int = 0) -> torch.Tensor:
        """Pinned host buffer [contrib_rows(B), W] the front door decodes into."""
        key = (B, slot)
        t = self._host_in.get(key)
        if t is None:
            t = self.layout.alloc(max(1, self.contrib_rows(B)), pin=self.cuda)
            self._host_in[key] = t
        return t

    def host_out(self, B: int, slot: int = 0) -> torch.Tensor:
        if self.scatter is not None:  # rank 0's shared output; rank r's share at r * B
            return self.scatter.out(slot)[: self.world * B]
        key = (B, slot)
        t = self._host_out.get(key)
        if t is None:
            t = torch.zeros(max(1, self.contrib_rows(B)), dtype=torch.float32, pin_memory=self.cuda)
            self._host_out[key] = t
        return t

    def step_out(self, B: int, slot: int = 0) -> torch.Tensor:
        """Where this rank's step writes its B scores."""
        if self.scatter is not None:
            return self.scatter.out(slot)[self.rank * B: (self.rank + 1) * B]
        return self.host_out(B, slot)[:B]

    def host_arena(self, slot: int = 0) -> torch.Tensor:
        """Pinned request arena of a slot (arena ingest)."""
        if self.scatter is not None:  # rank 0's batches live in the shared segment
            return self.scatter.arena(slot % self.scatter.n_arenas)
        t = self._host_arena.get(slot)
        if t is None:
            t = self._host_arena[slot] = self.arena.alloc(pin=self.cuda)
        return t

    def dev_arena(self, slot: int = 0) -> torch.Tensor:
        t = self._dev_arena.get(slot)
        if t is None:
            t = self._dev_arena[slot] = self.arena.alloc(device=self.dev)
        return t

    def _unpack(self, arena_dev: torch.Tensor, packed: torch.Tensor) -> None:
        from ..ops import hip

        self.arena.decode_varints(arena_dev)
        hip().unpack_arena(arena_dev, packed, self.layout.fields, self.layout.narrow_modulo)

    def _dev(self, store, key, shape, dtype):
        t = store.get(key)
        if t is None:
            t = torch.zeros(shape, dtype=dtype, device=self.dev)
            store[key] = t
        return t

    @property
    def lockstep(self) -> bool:
        """Every rank must launch every step (collectives inside the step):
        a candidate fan-out, or a model whose forward exchanges embeddings."""
        return self.mode != "local" or bool(getattr(self.ex.model, "has_collectives", False))

    def prepare(self, B: int) -> None:
        self.check_bucket(B)
        if self._program_enabled(B):
            if self._cprog is None and getattr(self.ex.model, "supports_program", False):
                from .native_comm import create_comm

                self._cprog = create_comm(self.ctx, self.group)
            for s in range(self.ex.slots):
                self.host_out(B, s)
                self._capture_program(B, s)
            self.program_active = True
            self._program_buckets.add(B)
            return
        native = self._native_fanout_enabled()
        if self.force_fanout and self.world == 1 and self.mode != "local" and not native:
            raise RuntimeError("force_fanout on one rank needs the native fan-out path (GPU + HIP graphs)")
        if native:
            self._ensure_comms()
        for s in range(self.ex.slots):
            if self.scatter is None:  # shared scatter: the batch stays in rank 0's shared arenas
                self.host_in(B, s)
            self.host_out(B, s)
            if self._step_graphs_enabled():
                self._capture_step(B, s)
            else:
                self.ex.prepare(B, s)
            if native:
                self._capture_ingress(B, s)
                self._capture_split(B, s)
        # a failed self-check disables the native path for good (every rank agreed)
        self.native_fanout_active = native and not self._native_disabled

    # -- programmed steps (embedding-parallel models) ------------------------------
    def _program_enabled(self, B: int) -> bool:
        if not (self.cuda and self.mode == "local" and self.native_launch and self.ingest == "arena"):
            return False
        # embedding-parallel models: the exchange is the program. Local
        # gather-GEMM steps can run as one too (DTFS_RESOLVE_LANE=1): the
        # resolve pass of step k+1 on the aux lane right after its H2D, the
        # compute lane waiting only for that - 108.4 vs 104.5 M scores/s with
        # round 4's 8-phase gather-GEMM (profiles/r04_session2.md). Off by
        # default since round 5: the one-wave gather-GEMM holds every
        # register of every SIMD, the aux lane's resolve cannot co-run (86 us
        # mean, starved) and the one-stream step measured 131.0 / 130.3 vs
        # 129.9 / 123.2 M interleaved (profiles/r05_gg1w.md).
        m = self.ex.model
        if getattr(m, "supports_program", False):
            return True
        if os.environ.get("DTFS_RESOLVE_LANE", "0") != "1" or not getattr(m, "resolve_lane", False):
            return False
        # only the buckets whose step runs the gather-GEMM (smaller steps keep
        # the one-stream step: no cross-lane hop on the light-load path)
        from ..ops import ArenaRows

        return bool(m._resolve_applies(ArenaRows(self.dev_arena(0), B, self.layout.fields), None))

    def _capture_program(self, B: int, slot: int) -> None:
        """Build and capture the step program of one (bucket, slot): GPU unpack
        of the request arena + the model's two-lane program, each kernel op
        captured into its own graph (parallel/step_program.py)."""
        from . import step_program as sp

        key = (B, slot)
        if key in self._programs:
            return
        model = self.ex.model
        buf = self.ex.input_buffer(B, slot)
        arena_dev = self.dev_arena(slot)
        h_out = self.host_out(B, slot)
        bufs = self._prog_bufs[key] = model.alloc(B) if hasattr(model, "alloc") else {}
        state: dict = {}
        if getattr(model, "supports_arena", False):
            # K0 fused: the program's kernels read ids / weights straight from
            # the request bytes (no unpack pass, no packed-row buffer)
            from ..ops import ArenaRows

            ops = [sp.Kernels(sp.AUX, lambda: self.arena.decode_varints(arena_dev), "varints")]
            ops += model.build_program(ArenaRows(arena_dev, B, self.layout.fields), None, B, bufs, out=h_out[:B],
                                       state=state)
        else:
            ops = [sp.Kernels(sp.AUX, lambda: self._unpack(arena_dev, buf), "unpack")]
            ops += model.build_program(self.layout.ids(buf), self.layout.wts(buf), B, bufs, out=h_out[:B],
                                       state=state)
        # warm-up: one eager run (collective on every rank, like the capture below)
        sp.run_eager(ops, self.group)
        torch.cuda.synchronize(self.dev)
        pools = {lane: torch.cuda.graph_pool_handle() for lane in (sp.COMPUTE, sp.AUX)}
        streams = {lane: torch.cuda.Stream(self.dev) for lane in (sp.COMPUTE, sp.AUX)}
        prog = sp.capture_native(ops, arena_dev, self._cprog, pools, streams, direct=True)
        prog.state = state  # the captured graphs' intermediate tensors live here
        self._programs[key] = prog

    def _launch_program(self, B: int, slot: int, h_in, h_out, rows: int, t0: float,
                        nbytes: Optional[int]) -> StepHandle:
        self._capture_program(B, slot)
        prog = self._programs[(B, slot)]
        self.runner().launch_program(slot, prog.spec, h_in, int(nbytes or 0))
        return StepHandle(B=B, slot=slot, host_out=h_out[:rows], event=_RunnerEvent(self._runner, slot, (self._cprog,)),
                          t_submit=t0, timeout_s=self.step_timeout_s)

    # -- native fan-out (world > 1) -----------------------------------------------
    def _native_fanout_enabled(self) -> bool:
        if self.scatter is not None:
            return False
        return (self.cuda and self.mode in ("alltoall", "scatter") and self.native_fanout and self.native_launch
                and self.ex.use_graphs and not getattr(self.ex.model, "has_collectives", False))

    def _ensure_comms(self) -> None:
        if self._cin is None:
            from .native_comm import create_comm

            # two communicators: the row exchange of step k+1 and the score
            # exchange of step k-1 run concurrently on different streams
            self._cin = create_comm(self.ctx, self.group)
            self._cout = create_comm(self.ctx, self.group)

    def _send_buf(self, B: int, slot: int) -> torch.Tensor:
        rows = self.contrib_rows(B)
        return self._dev(self._dev_send, (B, slot), (max(1, rows), self.layout.words), torch.int64)

    def _back_buf(self, B: int, slot: int) -> torch.Tensor:
        n = B if self.mode == "alltoall" else (self.world * B if self.rank == 0 else 1)
        return self._dev(self._dev_back, (B, slot), (n,), torch.float32)

    def _capture_ingress(self, B: int, slot: int) -> None:
        """Arena ingest: capture the GPU unpack (request bytes -> the slot's send
        rows) as a small graph the StepRunner launches on the ingress stream."""
        key = (B, slot)
        self._send_buf(B, slot)
        self._back_buf(B, slot)
        rows = self.contrib_rows(B)
        if self.ingest != "arena" or rows == 0 or key in self._ingress_graph:
            return
        arena_dev, send = self.dev_arena(slot), self._send_buf(B, slot)
        side = torch.cuda.Stream(self.dev)
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):
            self._unpack(arena_dev, send[:rows])
        side.synchronize()
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g, stream=side):
            self._unpack(arena_dev, send[:rows])
        g.instantiate()
        self._ingress_graph[key] = g

    def _capture_split(self, B: int, slot: int):
        """The fan-out step's two-lane forward: (resolve graph, rest-of-forward
        graph, scores) when the model's first layer is the gather-GEMM on these
        rows, else None. The StepRunner launches the resolve pass on the
        ingress lane right after the row exchange, so step k+1's resolve runs
        beside step k's gather-GEMM / tail on the compute lane - the local
        two-lane program's split (CTRModel.build_program) in fan-out form."""
        key = (B, slot)
        if key in self._split:
            return self._split[key]
        m = self.ex.model
        buf = self.ex.input_buffer(B, slot)
        ids, wts = self.layout.ids(buf), self.layout.wts(buf)
        res = None
        # off by default like the local program: 122.0 / 121.5 (on) vs 122.3 /
        # 123.0 M (off) interleaved with the one-wave gather-GEMM (profiles/r05_gg1w.md)
        if (self.cuda and self.ex.use_graphs and os.environ.get("DTFS_RESOLVE_LANE", "0") == "1"
                and getattr(m, "resolve_lane", False) and m._resolve_applies(ids, wts)):
            st: dict = {}
            side = torch.cuda.Stream(self.dev)
            side.wait_stream(torch.cuda.current_stream(self.dev))
            with torch.cuda.stream(side):  # warm-up (packs weights, allocates outside the capture)
                m._forward(ids, wts, resolved=m._resolve(ids, wts))
            side.synchronize()
            pool = torch.cuda.graph_pool_handle()
            g_res = torch.cuda.CUDAGraph(keep_graph=True)
            with torch.cuda.graph(g_res, pool=pool, stream=side):
                st["resolved"] = m._resolve(ids, wts)
            g_res.instantiate()
            g_fwd = torch.cuda.CUDAGraph(keep_graph=True)
            with torch.cuda.graph(g_fwd, pool=pool, stream=side):
                st["scores"] = m._forward(ids, wts, resolved=st["resolved"])
            g_fwd.instantiate()
            res = (g_res, g_fwd, st["scores"], st)
        self._split[key] = res
        return res

    def _forward_parts(self, B: int, slot: int):
        """(resolve graph or None, forward graph, device scores) of a fan-out step."""
        sp = self._capture_split(B, slot)
        if sp is not None:
            return sp[0], sp[1], sp[2]
        self.ex.prepare(B, slot)
        return None, self.ex._graphs[(B, slot)], self.ex._out[(B, slot)]

    def _launch_native_fanout(self, B: int, slot: int, h_in, h_out, rows: int, t0: float,
                              nbytes: Optional[int]) -> StepHandle:
        key = (B, slot)
        g_res, g_fwd, scores = self._forward_parts(B, slot)
        self._capture_ingress(B, slot)
        self.runner()
        send, back = self._send_buf(B, slot), self._back_buf(B, slot)
        if self.ingest == "arena":
            dst = self.dev_arena(slot)
            h2d = int(nbytes or 0) if rows else 0
        else:
            dst = send
            h2d = rows * self.layout.row_bytes
        ing = self._ingress_graph.get(key)
        self._runner.launch_fanout(
            slot, dst, h_in, h2d, ing.raw_cuda_graph_exec() if ing is not None else 0,
            self._cin, 0 if self.mode == "alltoall" else 1, send, self.ex.input_buffer(B, slot),
            g_fwd.raw_cuda_graph_exec(), self._cout, scores, back, h_out, rows * 4,
            g_res.raw_cuda_graph_exec() if g_res is not None else 0)
        return StepHandle(B=B, slot=slot, host_out=h_out[:rows], event=_RunnerEvent(self._runner, slot,
                                                                                   (self._cin, self._cout)),
                          t_submit=t0, timeout_s=self.step_timeout_s)

    def self_check(self, B: int, seed: int = 0, atol: float = 1e-5, slot: int = 0) -> bool:
        """Run one fan-out step on synthetic requests and compare every score
        with a local forward of the same candidate rows. With the native path
        active, a failure on ANY rank turns it off on every rank (eager
        torch.distributed path instead). Collective; returns the agreed result."""
        from ..client.synth import SyntheticRequests

        rows = self.contrib_rows(B)
        F = self.layout.fields
        ok = True
        err = ""
        try:
            synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=seed + 7919 * self.rank)
            ids = wts = None
            if rows:
                a_ids, a_wts = synth.arrays(rows)
                ids, wts = torch.from_numpy(a_ids), torch.from_numpy(a_wts)
            if rows and self.ingest == "arena":
                from ..ops import native

                reqs, per = [], 512
                for s in range(0, rows, per):
                    n = min(per, rows - s)
                    reqs.append(native().encode_predict_request(
                        "DCN", "serving_default", None,
                        [("feat_ids", ids[s:s + n].contiguous()), ("feat_wts", wts[s:s + n].contiguous())], True))
                ar = self.host_arena(slot)
                ab = self.arena.build(ar, self.arena.place(ar, reqs))
                h = self.launch(B, slot, src=ar, nbytes=ab.used_bytes)
            else:
                buf = self.host_in(B, slot)
                if rows:
                    self.layout.pack(ids, wts, out=buf[:rows])
                h = self.launch(B, slot, nbytes=0 if self.ingest == "arena" else None)
            got = h.wait().clone()
            if rows:
                want = self.ex.model(ids.to(self.dev), wts.to(self.dev)).float().cpu()
                diff = (got - want).abs().max().item()
                ok = bool(diff <= atol)
                err = f"max |diff| {diff:.3g}"
                # kept for the run's report (bench.py JSON "self_check")
                self.self_checks.append({"bucket": int(B), "rows": int(rows), "max_abs_diff": float(diff)})
        except Exception as e:  # surfaced through the agreement below
            ok, err = False, repr(e)
        if not ok:
            import sys

            print(f"[fanout] rank {self.rank}: self-check of bucket {B} failed: {err}", file=sys.stderr, flush=True)
        if self.ctx.is_distributed:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                                device=self.dev if self.ctx.backend == "nccl" else "cpu")
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
            all_ok = bool(flag.item())
        else:
            all_ok = ok
        if not all_ok and self.native_fanout_active:
            import sys

            print(f"[fanout] rank {self.rank}: native fan-out self-check failed ({err or 'on another rank'}); "
                  f"using the torch.distributed path", file=sys.stderr, flush=True)
            self.native_fanout_active = False
            self._native_disabled = True
            if self.cuda:
                torch.cuda.synchronize(self.dev)
        return all_ok

    def runner(self):
        """The native StepRunner of this engine's device (created on first use)."""
        if self._runner is None:
            from ..ops import hip

            self._runner = hip().StepRunner(self.dev.index if self.dev.index is not None else 0, self.ex.slots)
        return self._runner

    def loop_slots(self, B: int):
        """Per-slot launch descriptions for the GPU live server
        (csrc/runtime/step_runner.h LoopSlot): a local step, a fan-out step or a
        programmed step."""
        if not self.cuda or self.ingest != "arena":
            raise RuntimeError("the native serving loop needs a GPU and arena ingest")
        from ..ops import hip

        self.prepare(B)

        # direct kernel launches instead of hipGraphLaunch (runtime/kernel_seq.h:
        # ~8-14 us less idle per step)
        def seq(g):
            if g is None:
                return None
            k = id(g)
            if k not in self._seqs:
                try:
                    self._seqs[k] = hip().KernelSequence(g.raw_cuda_graph())
                except RuntimeError:  # a node type the sequence cannot replay: keep the graph
                    self._seqs[k] = None
            return self._seqs[k]

        out = []
        rows = self.contrib_rows(B)
        for s in range(self.ex.slots):
            h_out = self.host_out(B, s)
            if B in self._program_buckets:
                self._capture_program(B, s)
                out.append(dict(program=self._programs[(B, s)].spec, h2d_dst=self.dev_arena(s), h_out=h_out))
            elif self._step_graphs_enabled():
                self._capture_step(B, s)
                g = self._step_graph[(B, s)]
                out.append(dict(h2d_dst=self.dev_arena(s), graph_exec=g.raw_cuda_graph_exec(), seq=seq(g),
                                h_out=h_out))
            elif self.native_fanout_active:
                key = (B, s)
                g_res, fwd, scores = self._forward_parts(B, s)
                self._capture_ingress(B, s)
                ing = self._ingress_graph.get(key)
                out.append(dict(
                    fanout=True, h2d_dst=self.dev_arena(s),
                    ingress_exec=ing.raw_cuda_graph_exec() if ing is not None else 0, ingress_seq=seq(ing),
                    cin=self._cin, cout=self._cout, mode=0 if self.mode == "alltoall" else 1,
                    send=self._send_buf(B, s), recv=self.ex.input_buffer(B, s),
                    forward_exec=fwd.raw_cuda_graph_exec(), forward_seq=seq(fwd), scores=scores,
                    resolve_exec=g_res.raw_cuda_graph_exec() if g_res is not None else None,
                    resolve_seq=seq(g_res), back=self._back_buf(B, s), h_out=h_out, d2h_bytes=rows * 4))
            else:
                raise RuntimeError("no native step path for this engine (graphs disabled or fan-out fell back)")
        return out

    def comm_error(self) -> Optional[str]:
        """Asynchronous RCCL error of the native communicators (failure detection)."""
        from .native_comm import check_comms

        return check_comms(self._cin, self._cout, self._cprog)

    def abort(self) -> None:
        """Abort the native communicators (a peer is gone / a deadline passed)."""
        for c in (self._cin, self._cout, self._cprog):
            if c is not None:
                c.abort()

    # -- whole-step graphs (no fan-out) ------------------------------------------
    def _step_graphs_enabled(self) -> bool:
        return (self.cuda and (self.mode == "local" or self.scatter is not None) and self.ex.use_graphs
                and self.step_graphs)

    def _capture_step(self, B: int, slot: int) -> None:
        """Capture forward -> D2H of one (bucket, slot) as ONE HIP graph.

        The H2D is deliberately NOT in the graph: inside a graph ROCm turns a
        memcpy node into a blit kernel that competes with the GEMMs for CUs
        (measured: both slowed ~2x), while an eager pinned H2D on its own stream
        runs on an SDMA engine and overlaps the previous step's kernels for free.
        All compute stays on one stream: two forwards sharing the chip only
        thrash each other's L2."""
        key = (B, slot)
        if key in self._step_graph:
            return
        cur = torch.cuda.current_stream(self.dev)
        out = self.step_out(B, slot)
        buf = self.ex.input_buffer(B, slot)
        arena_dev = self.dev_arena(slot) if self.ingest == "arena" else None

        fused_ingest = arena_dev is not None and getattr(self.ex.model, "supports_arena", False)

        def body():
            # the head kernel writes the scores straight into pinned host memory
            # (no D2H copy node, which a graph would run as a blit kernel)
            if fused_ingest:  # K0 fused into K1: the gather reads the request bytes
                self.arena.decode_varints(arena_dev)
                self.ex.model.forward_arena(arena_dev, B, out=out)
                return
            if arena_dev is not None:  # K0 on the GPU: request bytes -> packed rows
                self._unpack(arena_dev, buf)
            self.ex._forward(buf, out=out)

        side = torch.cuda.Stream(self.dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(2):
                body()
        side.synchronize()
        pool = self.ex._pools.get(("step", slot))
        if pool is None:
            pool = self.ex._pools[("step", slot)] = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph(keep_graph=True)  # the native loop replays its nodes directly
        with torch.cuda.graph(g, pool=pool, stream=side):
            body()
        g.instantiate()
        self._step_graph[key] = g

    def _launch_step_graph(self, B: int, slot: int, h_in, h_out, rows: int, t0: float,
                           nbytes: Optional[int] = None) -> StepHandle:
        self._capture_step(B, slot)
        # H2D target: the graph's packed-row input, or (arena ingest) the slot's device arena
        dst = self.dev_arena(slot) if self.ingest == "arena" else self.ex.input_buffer(B, slot)
        if nbytes is None:
            nbytes = B * self.layout.row_bytes
        if self.native_launch:
            # C++ StepRunner: SDMA H2D + hipGraphLaunch + events, no torch stream
            # bookkeeping in the loop (csrc/runtime/step_runner.cpp)
            self.runner().launch(slot, dst, h_in, nbytes, self._step_graph[(B, slot)].raw_cuda_graph_exec())
            return StepHandle(B=B, slot=slot, host_out=h_out[:rows], event=_RunnerEvent(self._runner, slot),
                              t_submit=t0, timeout_s=self.step_timeout_s)
        cur = torch.cuda.current_stream(self.dev)
        ev_in_free = self._ev_in_free.get(slot)
        with torch.cuda.stream(self.h2d_stream):  # SDMA, overlaps the previous step
            if ev_in_free is not None:
                self.h2d_stream.wait_event(ev_in_free)
            dst.view(-1)[: nbytes // dst.element_size()].copy_(
                h_in.view(-1)[: nbytes // h_in.element_size()], non_blocking=True)
        cur.wait_stream(self.h2d_stream)
        self._step_graph[(B, slot)].replay()
        ev = torch.cuda.Event()
        ev.record(cur)
        self._ev_in_free[slot] = ev
        return StepHandle(B=B, slot=slot, host_out=h_out[:rows], event=ev, t_submit=t0, timeout_s=self.step_timeout_s)

    # -- one step --------------------------------------------------------------
    def launch(self, B: int, slot: int = 0, src: Optional[torch.Tensor] = None,
               nbytes: Optional[int] = None) -> StepHandle:
        """Enqueue one fan-out step for bucket B.

        Input: host_in(B, slot) packed rows, or with arena ingest the request
        arena ``src`` (default host_arena(slot)) of which ``nbytes`` are used.
        Returns immediately on GPU (all work is stream-ordered); call
        ``handle.wait()`` for the scores in host_out(B, slot)."""
        self.check_bucket(B)
        key = (B, slot)
        h_out = self.host_out(B, slot)
        arena_mode = self.ingest == "arena"
        if arena_mode:
            h_in = self.host_arena(slot) if src is None else src
            if nbytes is None:
                raise ValueError("arena ingest: pass nbytes (ArenaBatch.used_bytes)")
        else:
            h_in = self.host_in(B, slot) if src is None else src
        rows = self.contrib_rows(B)
        t0 = time.perf_counter()
        exec_in = self.ex.input_buffer(B, slot)
        if not self.cuda and self.scatter is not None:
            return self._launch_shared_scatter_cpu(B, slot, h_in, h_out, rows, exec_in, t0)
        if not self.cuda:
            if arena_mode:  # host reference of the GPU unpack
                packed = self.host_in(B, slot)
                if rows:
                    if self.layout.narrow:  # wide unpack, then the narrow row form
                        from ..serving.packing import PackedLayout

                        wide = PackedLayout(self.layout.fields)
                        tmp = self.arena.unpack_cpu(h_in, wide.alloc(rows))
                        self.layout.pack(wide.ids(tmp), wide.wts(tmp), out=packed[:rows])
                    else:
                        self.arena.unpack_cpu(h_in, packed[:rows])
                h_in = packed
            return self._launch_cpu(B, slot, h_in, h_out, rows, exec_in, t0)
        if B in self._program_buckets:
            return self._launch_program(B, slot, h_in, h_out, rows, t0, nbytes)
        if self.scatter is not None:
            return self._launch_shared_scatter(B, slot, h_in, h_out, rows, t0)
        if self._step_graphs_enabled():
            return self._launch_step_graph(B, slot, h_in, h_out, rows, t0, nbytes)
        if self.native_fanout_active:
            return self._launch_native_fanout(B, slot, h_in, h_out, rows, t0, nbytes)

        cur = torch.cuda.current_stream(self.dev)
        ev_in_free = self._ev_in_free.get(slot)
        ev_out_free = self._ev_out_free.get(slot)
        # H2D: straight into the executor's graph input when there is no fan-out
        if self.mode == "local":
            send = exec_in
        else:
            send = self._dev(self._dev_send, key, (max(1, rows), self.layout.words), torch.int64)
        with torch.cuda.stream(self.h2d_stream):
            # WAR: wait only until this slot's previous step has consumed its
            # input, so this H2D overlaps the previous step's compute
            if ev_in_free is not None:
                self.h2d_stream.wait_event(ev_in_free)
            if rows and arena_mode:
                ad = self.dev_arena(slot)
                ad[:nbytes].copy_(h_in[:nbytes], non_blocking=True)
            elif rows:
                send[:rows].copy_(h_in[:rows], non_blocking=True)
        cur.wait_stream(self.h2d_stream)
        if rows and arena_mode:
            self._unpack(self.dev_arena(slot), send[:rows])

        if self.mode == "alltoall":
            dist.all_to_all_single(exec_in, send, group=self.group)
        elif self.mode == "scatter":
            chunks = list(send[: self.world * B].chunk(self.world)) if self.rank == 0 else None
            dist.scatter(exec_in, chunks, src=0, group=self.group)
        if self.mode != "local":
            ev = torch.cuda.Event()
            ev.record(cur)
            self._ev_in_free[slot] = ev

        if ev_out_free is not None:  # WAR on this slot's graph output / back buffer
            cur.wait_event(ev_out_free)
        scores = self.ex.run(B, slot)
        if self.mode == "local":
            ev = torch.cuda.Event()
            ev.record(cur)
            self._ev_in_free[slot] = ev

        if self.mode == "alltoall":
            back = self._dev(self._dev_back, key, (B,), torch.float32)
            dist.all_to_all_single(back, scores, group=self.group)
        elif self.mode == "scatter":
            back = self._dev(self._dev_back, key, (self.world * B,), torch.float32) if self.rank == 0 else None
            dist.gather(scores, list(back.chunk(self.world)) if self.rank == 0 else None, dst=0, group=self.group)
        else:
            back = scores

        done = torch.cuda.Event()
        with torch.cuda.stream(self.d2h_stream):
            self.d2h_stream.wait_stream(cur)
            if rows:
                h_out[:rows].copy_(back[:rows], non_blocking=True)
            done.record(self.d2h_stream)
        self._ev_out_free[slot] = done
        return StepHandle(B=B, slot=slot, host_out=h_out[:rows], event=done, t_submit=t0, timeout_s=self.step_timeout_s)

    # -- shared-arena scatter ----------------------------------------------------
    def _launch_shared_scatter(self, B: int, slot: int, h_in, h_out, rows: int, t0: float) -> StepHandle:
        """One step on this rank's share of rank 0's shared batch (GPU): the
        native StepRunner copies the share and launches the captured local
        step (csrc/bindings_hip.cpp scatter_step)."""
        self._capture_step(B, slot)
        g = self._step_graph[(B, slot)]
        k = self.scatter.launch(self.runner(), slot, B, h_in if self.rank == 0 else None, self.dev_arena(slot), None,
                                g.raw_cuda_graph_exec(), self.step_timeout_s or 30.0)
        return StepHandle(B=B, slot=slot, host_out=h_out[:rows], event=_ScatterEvent(self, slot, k), t_submit=t0,
                          timeout_s=self.step_timeout_s)

    def _launch_shared_scatter_cpu(self, B, slot, h_in, h_out, rows, exec_in, t0) -> StepHandle:
        """Host reference of the shared-arena scatter step (CPU ranks, gloo
        tests): the same plan and share copies (memcpy instead of DMA) into a
        private arena, the local forward, scores into rank 0's shared output."""
        seg = self.scatter
        timeout = self.step_timeout_s or 30.0
        k = seg.begin_step()
        if self.rank == 0:
            ai = seg.arena_index(h_in)
            if ai < 0:
                raise RuntimeError("shared scatter: rank 0's batch is not in a shared arena")
            seg.publish_plan(k, ai, B)
        local = self._local_arena.get(slot)
        if local is None:
            local = self._local_arena[slot] = self.arena.alloc()
        row0, n, _ = seg.take_share(k, local, timeout)
        packed = self.layout.alloc(B)
        self.arena.unpack_cpu(local, packed)
        exec_in[:B].copy_(packed[:B])
        scores = self.ex.run(B, slot).contiguous()
        if n:  # the rank's fixed slice, as the GPU step's captured head writes it
            self.step_out(B, slot)[:n].copy_(scores[:n])
        seg.mark_done(k)
        if self.rank == 0:
            ok, err = seg.wait_done(k, timeout)
            if not ok:
                raise StepTimeout(f"shared scatter step failed: {err}")
            seg.compact_scores(k, slot)
        return StepHandle(B=B, slot=slot, host_out=h_out[:rows], event=None, t_submit=t0)

    def _launch_cpu(self, B, slot, h_in, h_out, rows, exec_in, t0) -> StepHandle:
        if self.mode == "alltoall":
            dist.all_to_all_single(exec_in, h_in[:B].contiguous(), group=self.group)
        elif self.mode == "scatter":
            chunks = list(h_in[: self.world * B].chunk(self.world)) if self.rank == 0 else None
            dist.scatter(exec_in, chunks, src=0, group=self.group)
        else:
            exec_in[:B].copy_(h_in[:B])
        scores = self.ex.run(B, slot).contiguous()
        if self.mode == "alltoall":
            back = torch.empty(B, dtype=torch.float32)
            dist.all_to_all_single(back, scores, group=self.group)
        elif self.mode == "scatter":
            back = torch.empty(self.world * B, dtype=torch.float32) if self.rank == 0 else None
            dist.gather(scores, list(back.chunk(self.world)) if self.rank == 0 else None, dst=0, group=self.group)
        else:
            back = scores
        if rows:
            h_out[:rows].copy_(back[:rows])
        return StepHandle(B=B, slot=slot, host_out=h_out[:rows], event=None, t_submit=t0)
