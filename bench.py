"""Benchmark: device-resident Bloom probes/s on the C3 workload (BASELINE.json).

One step = one batched multi-filter probe of 1M 16-byte lookup keys (already
in HBM) against this GPU's 32 resident 8-MiB filters (m = 2^26), producing the
[filter][n/64] hit bitmaps; for N > 1 GPUs each rank holds its own 32 filters
(filters shard one subset per GPU, weak scaling) and the step also all-gathers
the hit bitmaps over RCCL/xGMI. value = probes of all ranks / max-rank time.

Also reported (same JSON line): C2 build keys/s (1M keys -> one 16 MiB filter),
the dominant kernel's roofline (HIP events on its own stream), the CPU oracle
baseline (rank 0, N = 1), and the PCIe-inclusive end-to-end probe rate.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment) starts
the N rank processes itself through torch.distributed.run before anything
touches the GPU, and relays rank 0's JSON line; inside a rank, --gpus must
equal WORLD_SIZE. --dry-run joins a gloo group and reports every rank's
RANK / LOCAL_RANK / WORLD_SIZE without any GPU call (the launcher's CPU test).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Bloom probes/sec device-resident (1M keys × 32 filters); build keys/sec"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--workload", choices=["c3", "c4", "c5"], default="c3",
                   help="c3: 1M keys x 32 filters/GPU probe (default, the BASELINE metric); "
                        "c5: 10M keys x 32 filters/GPU probe; c4: 64 concurrent builds of 256K keys "
                        "(m=2^25) split over the GPUs")
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--leg-steps", type=int, default=200,
                   help="steps of each secondary leg (build, read path, zone, flush/4, rotating, one lane): "
                        "at least --steps; the headline leg times exactly --steps")
    p.add_argument("--n-keys", type=int, default=None,
                   help="lookup keys per step (default: 2^20 for c3, 10,000,000 for c5)")
    p.add_argument("--filters", type=int, default=32, help="filters per GPU")
    p.add_argument("--m-bits", type=int, default=1 << 26)
    p.add_argument("--keys-per-filter", type=int, default=1 << 19)
    p.add_argument("--build-keys", type=int, default=1 << 20)
    p.add_argument("--build-m-bits", type=int, default=1 << 27)
    p.add_argument("--path", type=int, default=0, help="0 auto, 1 direct, 2 tiled")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU oracle baseline")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--check", action="store_true", help="verify hits against the oracle (slow)")
    p.add_argument("--no-zone", action="store_true", help="skip the zone-map gate leg (and the read path)")
    p.add_argument("--no-read", action="store_true", help="skip the SSTable read-path leg")
    p.add_argument("--no-flush", action="store_true", help="skip the flush-producer (SsTable::create) leg")
    p.add_argument("--no-cold", action="store_true",
                   help="skip the cold-cache legs (profiles: keeps every k_set_probe launch warm, so "
                        "rocprofv3's average matches the bench line's warm kernel time)")
    p.add_argument("--no-c4", action="store_true", help="skip the C4 leg (64 concurrent builds) of the default line")
    p.add_argument("--no-c5", action="store_true", help="skip the C5 rank-slice leg (10M keys x 32 filters)")
    p.add_argument("--no-wide", action="store_true",
                   help="skip the wide fan-out leg (300 auto-flush-sized tables of m=1024 in one wide set)")
    p.add_argument("--flush-entries", type=int, default=1 << 20)
    p.add_argument("--build-streams", type=int, default=4, choices=[1, 2, 3, 4],
                   help="pipeline lanes of the C2 build leg (independent flushes in flight)")
    p.add_argument("--probe-streams", type=int, default=3, choices=[1, 2, 3, 4],
                   help="pipeline lanes: consecutive steps alternate over this many streams (each with "
                        "its own hit buffers; for N > 1 they share the rank's one RCCL communicator)")
    p.add_argument("--force-dist", action="store_true",
                   help="initialise the process group and run the exchange path even at N=1")
    p.add_argument("--set-dense", choices=["auto", "on", "off"], default="auto",
                   help="FilterSet probes of dense batches (cb_set_dense): auto = the region-partitioned "
                        "probe when a batch holds >= 2 keys per 128-B set line (C5), on / off = always / never")
    p.add_argument("--leg", choices=["c2", "c5", "wide"], default=None,
                   help="run only that secondary leg (the C2 build, the C5 rank slice, or the wide fan-out) and print one "
                        "line holding it: the rocprofv3 passes of tools/profile_round.sh, so the trace and the "
                        "counters hold that leg's kernels alone")
    p.add_argument("--full-line", default=None, metavar="PATH",
                   help="also write the full (uncompacted) JSON line, with every leg's prose fields, to PATH; stdout "
                        "carries the compact line (compact_line: <= 8 KB, the legs the driver's tail must show last)")
    p.add_argument("--phase-deadline", type=float, default=120.0,
                   help="per-rank watchdog: seconds a guarded phase (rendezvous, RCCL init, each timed region and "
                        "its warm-up, each check's collective) may take before the rank aborts its communicator, "
                        "prints one JSON diagnostic line to stderr and exits 4")
    p.add_argument("--job-deadline", type=float, default=1200.0,
                   help="`--gpus N` parent: seconds the N ranks may take in all before it kills them and exits 5")
    p.add_argument("--dry-run", action="store_true",
                   help="launch / join the ranks over gloo and report them; no GPU work")
    p.add_argument("--rehearse-one-gpu", action="store_true",
                   help="run the N-rank path with every rank on GPU 0: gloo process group and the C ABI's "
                        "host transport (cb_comm_init_host) instead of RCCL; checks the multi-rank flow on a "
                        "one-GPU box, its numbers are not a scaling measurement")
    a = p.parse_args()
    if a.n_keys is None:
        a.n_keys = 10_000_000 if a.workload == "c5" else 1 << 20
    return a


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher: start N fresh rank processes
    (python -m torch.distributed.run, one per GPU, rendezvous on 127.0.0.1)
    running this same command line, relay rank 0's JSON line to stdout, and
    return the launcher's exit status (non-zero when any rank failed). The
    parent never imports torch or touches HIP: each rank initialises its own
    GPU.

    Failure bound: a rank whose guarded phase outlives
    --phase-deadline aborts its communicator and exits 4 (Watchdog), and
    torch.distributed.run then ends the other ranks and fails; as a backstop,
    when the whole job outlives --job-deadline the parent kills the launcher's
    process group (every rank) and exits 5, printing one JSON diagnostic line
    to stderr."""
    import signal
    import socket
    import threading
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, CB_BENCH_LAUNCHER="bench.py")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL over dmabuf IPC on this host driver
    log(f"[launcher] {args.gpus} ranks: {' '.join(cmd)}")
    t0 = time.monotonic()
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, start_new_session=True)
    out = []

    def relay():
        for line in p.stdout:  # the ranks' stderr is inherited (progress stays visible)
            if line.lstrip().startswith("{"):
                out.append(line.strip())
            elif line.strip():
                log(line.rstrip())

    reader = threading.Thread(target=relay, daemon=True)
    reader.start()
    try:
        rc = p.wait(timeout=args.job_deadline)
    except subprocess.TimeoutExpired:
        log(json.dumps({"error": "job deadline", "seconds": round(time.monotonic() - t0, 1),
                        "job_deadline": args.job_deadline, "n_ranks": args.gpus,
                        "action": "killed the launcher's process group (every rank)"}))
        for sig, wait in ((signal.SIGTERM, 10), (signal.SIGKILL, 10)):
            try:
                os.killpg(p.pid, sig)
            except ProcessLookupError:
                break
            try:
                p.wait(timeout=wait)
                break
            except subprocess.TimeoutExpired:
                continue
        return 5
    reader.join(timeout=10)
    if rc == 0 and len(out) != 1:
        log(f"[launcher] error: expected one JSON line from rank 0, got {len(out)}")
        return 1
    if rc == 0:
        print(out[0], flush=True)
    else:
        log(f"[launcher] a rank failed (exit status {rc}); no result line")
    return rc


class Watchdog:
    """A rank's failure bound (Next 3): the first N > 1 RCCL run
    must not spend the driver's whole timeout on a hang at init or in a
    collective. Guarded phases (`with guard("name"):`) each get
    --phase-deadline seconds; a daemon thread checks the clock, and when a
    phase outlives it the rank aborts its library communicator
    (cb_comm_abort = ncclCommAbort, which also ends a collective another
    thread is blocked in), prints one JSON line {"error": "deadline", rank,
    phase, seconds, rccl_world} to stderr and leaves with os._exit(4) (no
    re-exec, no cleanup that could block on the device).
    CB_BENCH_STALL="RANK:PHASE" makes that rank stall inside that phase (the
    CPU test of the bound)."""

    def __init__(self, rank: int, world: int, seconds: float):
        import threading
        self.rank, self.world, self.seconds = rank, world, seconds
        self.comm = None
        self._lock = threading.Lock()
        self._phase, self._until, self._t0 = None, None, None
        stall = os.environ.get("CB_BENCH_STALL", "")
        self._stall = tuple(stall.split(":", 1)) if ":" in stall else None
        threading.Thread(target=self._watch, daemon=True).start()

    def guard(self, phase: str, seconds: float | None = None):
        import contextlib

        @contextlib.contextmanager
        def cm():
            with self._lock:
                outer = (self._phase, self._until, self._t0)
                self._phase = phase
                self._t0 = time.monotonic()
                self._until = self._t0 + (seconds or self.seconds)
            try:
                if self._stall == (str(self.rank), phase):
                    log(f"[rank {self.rank}] CB_BENCH_STALL: stalling in phase {phase}")
                    while True:
                        time.sleep(1)
                yield
            finally:
                with self._lock:
                    self._phase, self._until, self._t0 = outer
        return cm()

    def _watch(self):
        while True:
            time.sleep(0.25)
            with self._lock:
                late = self._until is not None and time.monotonic() > self._until
                phase, t0 = self._phase, self._t0
            if late:
                self._fire(phase, time.monotonic() - t0)

    def _fire(self, phase, took):
        rc = None
        cw = None
        if self.comm is not None:
            cw = getattr(self.comm, "world", None)
            try:
                rc = self.comm.abort()
            except Exception as e:  # the diagnostic must still go out
                rc = repr(e)
        sys.stderr.write(json.dumps({"error": "deadline", "rank": self.rank, "world": self.world, "phase": phase,
                                     "seconds": round(took, 1), "phase_deadline": self.seconds,
                                     "rccl_world": cw, "comm_abort": rc}) + "\n")
        sys.stderr.flush()
        os._exit(4)


_WD = None  # this rank's Watchdog


def guard(phase: str, seconds: float | None = None):
    """A guarded phase of this rank (Watchdog), or a no-op without one."""
    import contextlib
    return _WD.guard(phase, seconds) if _WD is not None else contextlib.nullcontext()


def dry_run(args, world, rank, local, result) -> None:
    """Join the ranks over gloo and report each one's identity (no GPU)."""
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    with guard("rendezvous", 5 * args.phase_deadline):
        dist.init_process_group("gloo", rank=rank, world_size=world)
    me = {"rank": rank, "local_rank": local, "world_size": int(os.environ.get("WORLD_SIZE", "1")),
          "pid": os.getpid()}
    every = [None] * world
    with guard("dry_run"):
        dist.all_gather_object(every, me)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "gpus_arg": args.gpus,
                          "launcher": os.environ.get("CB_BENCH_LAUNCHER", "external"), "ranks": every}),
              file=result, flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))  # before anything touches the GPU
    # The contract is ONE JSON line on stdout. Libraries (RCCL's banner, ...)
    # write to fd 1 directly, so fd 1 is pointed at stderr for the whole run
    # and the result line goes to a saved copy of the original stdout.
    out_fd = os.dup(1)
    os.dup2(2, 1)
    result = os.fdopen(out_fd, "w")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world}: run `bench.py --gpus N` alone (it starts the N "
            "ranks) or under a launcher with --nproc-per-node N")
        sys.exit(2)
    global _WD
    if world > 1 or args.force_dist:
        _WD = Watchdog(rank, world, args.phase_deadline)
    if args.dry_run:
        return dry_run(args, world, rank, local, result)
    import torch
    import torch.distributed as dist

    rehearse = args.rehearse_one_gpu
    local_rank = local
    if rehearse:
        local = 0  # every rank on GPU 0 (the one-GPU rehearsal of the N-rank path)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_dist = world > 1 or args.force_dist
    if use_dist:
        if "MASTER_ADDR" not in os.environ:
            os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", "29533"
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        # ONE RCCL communicator per GPU: the library's own (cb_comm, the hit
        # exchange, created below from a 128-byte id). torch.distributed is
        # only the launcher's rendezvous, the barriers at the timed regions'
        # edges and the max-over-ranks timing, all host-side, so its process
        # group is gloo on every path (no second NCCL/RCCL communicator on the
        # device, no torch collective that could interleave with the library's
        # on a GPU stream). Every barrier follows a device synchronize.
        # (the ranks reach the rendezvous at different times: the first
        # `import torch` on a fresh box can take 1-2 minutes, so this phase
        # gets five times the deadline)
        with guard("rendezvous", 5 * args.phase_deadline):
            dist.init_process_group("gloo")
    # host-side reductions (timing max, check flags) run on the CPU (gloo)
    red_dev = torch.device("cpu")
    log(f"[rank {rank}] local rank {local_rank} on cuda:{local} of world {world}")

    import lsmt_amd
    from lsmt_amd import _lib, workload
    from lsmt_amd.shard import Comm, shard_range, sparse_cap

    L = _lib.load()
    lsmt_amd.set_path(args.path)
    lsmt_amd.set_dense({"auto": 0, "on": 1, "off": -1}[args.set_dense])
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    if args.workload == "c4":
        return run_c4(args, torch, dist, world, rank, local, dev, use_dist, result, red_dev)
    if args.leg:
        return run_leg(args, torch, dist, world, rank, local, dev, use_dist, result, red_dev)
    seed_base, absent_seed = 100, 999
    if args.workload == "c5":  # key(1000+f, i), absent key(9999, i)
        seed_base, absent_seed = 1000, 9999
    F, n, m, kpf = args.filters, args.n_keys, args.m_bits, args.keys_per_filter
    nf_total = F * world  # weak scaling: F filters per GPU
    f_lo, f_hi = shard_range(nf_total, world, rank)
    assert f_hi - f_lo == F

    # ---- setup (untimed): build this rank's filters, stage the lookups in HBM
    t_setup = time.time()
    filters = []
    for f in range(f_lo, f_lo + F):
        keys = torch.from_numpy(workload.key_range(seed_base + f, kpf)).to(dev)
        b = lsmt_amd.BloomFilter(m, device=local)
        b.insert_batch(lsmt_amd.DeviceKeys(keys), stream=sh)
        filters.append(b)
    look_np = workload.probe_lookups(n, nf_total, kpf, seed_base=seed_base, absent_seed=absent_seed)
    look = torch.from_numpy(look_np).to(dev)
    words = (n + 63) // 64
    # one hit buffer (and one gathered map) per pipeline lane (below)
    hits_bufs = [torch.zeros((F, words), dtype=torch.int64, device=dev) for _ in range(args.probe_streams)]
    hits_all_bufs = [torch.zeros((nf_total, words), dtype=torch.int64, device=dev)
                     for _ in range(args.probe_streams)] if use_dist else hits_bufs
    step_no = [0]
    torch.cuda.synchronize(dev)
    log(f"[rank {rank}] setup {time.time() - t_setup:.1f}s: {F} filters m={m} built, {n} lookups in HBM")
    keys_batch = lsmt_amd.DeviceKeys(look)

    # FilterSet: the same F filters bit-sliced ([m][F]); built once from the
    # filters (a full transpose) and timed separately as a maintenance cost.
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    fset = lsmt_amd.FilterSet(m, width=32 if F <= 32 else 64, device=local)
    fset.assign_all(filters, stream=sh)
    torch.cuda.synchronize(dev)
    set_build_ms = (time.perf_counter() - t0) * 1e3

    # Sparse exchange (cb_hits_allgather, CB_XCHG_SPARSE): ship set-bit
    # positions instead of dense rows. Default whenever a pack is under half
    # the dense rows (every N >= 2 at C3: 1.5 MB vs 4 MiB per rank at N = 2,
    # 0.5 MB vs 4 MiB at N = 8), since xGMI is point-to-point and the bytes a
    # rank receives bound the all-gather, while compress + expand cost ~12 us
    # on the device (profiles/xchg_*_r02); CB_SPARSE_EXCHANGE=1/0 forces it.
    from lsmt_amd.shard import pack_words
    sparse_env = os.environ.get("CB_SPARSE_EXCHANGE")
    cap = sparse_cap(n, nf_total, world)
    pack_bytes = 4 * pack_words(F * words, cap)
    use_sparse = use_dist and (sparse_env == "1" or (sparse_env != "0" and world >= 2 and
                                                     2 * pack_bytes < 8 * F * words))
    xstats = {"sparse_steps": 0}
    # asynchronous overflow report (no host round trip per step): cleared by
    # k_hits_expand if any rank's set bits ever exceed cap; checked below
    # before the results are reported
    x_ok = torch.ones(1, dtype=torch.int32, device=dev) if use_sparse else None

    # Pipelined batches: consecutive steps go round-robin to P "lanes", each
    # with its own HIP stream, hit buffers and (N > 1) RCCL communicator, so
    # one batch's launch ramp, drain and exchange overlap the next batch's
    # probe. A step is still one full probe (+ exchange) of one batch; lanes
    # never share a buffer, so no cross-stream event is needed per step.
    P = args.probe_streams
    # every lane stream the line will use (the probe lanes first, then the
    # build's extra ones), made together at its start (leg_lanes)
    all_lanes = [stream] + [torch.cuda.Stream(device=dev) for _ in range(max(P, args.build_streams) - 1)]
    lane_streams = all_lanes[:P]
    global _LANES
    _LANES = all_lanes
    lane_sh = [st.cuda_stream for st in lane_streams]
    # The exchange runs through the C ABI (cb_hits_allgather over the
    # library's own RCCL communicator, lsmt_amd/csrc/comm.cpp): the same call
    # a Rust Database::get would make. torch.distributed only hands out the
    # communicator id and times the run. ONE communicator per rank, shared by
    # the lanes: the library keeps each lane's packs apart and runs the
    # collectives in issue order (every rank issues them in the same order),
    # so no two collectives are ever in flight at once.
    if use_dist and rehearse:
        def gloo_allgather(send, recv):
            nb = send.size
            parts = [torch.empty(nb, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(send.copy()))
            for r, part in enumerate(parts):
                recv[r * nb:(r + 1) * nb] = part.numpy()

        with guard("comm_init"):
            xcomm = Comm.host(rank, world, local, gloo_allgather)
    else:
        with guard("rccl_init", 2 * args.phase_deadline):
            xcomm = Comm.from_process_group(local) if use_dist else None
    if _WD is not None:
        _WD.comm = xcomm
    if xcomm is not None and xcomm.world != world:
        raise RuntimeError(f"RCCL communicator has {xcomm.world} ranks, WORLD_SIZE is {world}")
    # every rank's own view of its communicator's world (the line's
    # rccl_world: one entry per rank, each the library's cb_comm_info)
    rccl_world = None
    if use_dist:
        every = [None] * world
        with guard("rccl_world"):
            dist.all_gather_object(every, xcomm.world)
        rccl_world = every

    def exchange(buf):
        """All-gather this step's hit rows from every rank (filter-major ->
        plain concatenation) over RCCL/xGMI, on the step's lane right after
        its probe."""
        if not use_dist:
            return
        if use_sparse:
            xcomm.allgather(hits_bufs[buf], nf_total, hits_all_bufs[buf], sparse=True, cap=cap,
                            ok=x_ok, stream=lane_sh[buf])
            xstats["sparse_steps"] += 1
        else:
            xcomm.allgather(hits_bufs[buf], nf_total, hits_all_bufs[buf], stream=lane_sh[buf])

    def claim():
        buf = step_no[0] % P
        step_no[0] += 1
        return buf

    def step_tiled():
        buf = claim()
        lsmt_amd.probe(filters, keys_batch, out=hits_bufs[buf], stream=lane_sh[buf])
        exchange(buf)

    def set_step(buf, gated=False):
        """One FilterSet step. N > 1: the probe and the exchange are one C call
        (cb_set_probe_allgather_fixed): in sparse mode the probe kernel writes
        the pack itself, so no separate compress pass reads the rows again."""
        if use_dist:
            xcomm.probe_allgather(fset, look, nf_total, hits_bufs[buf], hits_all_bufs[buf], sparse=use_sparse,
                                  cap=cap, ok=x_ok, gated=gated, stream=lane_sh[buf])
            xstats["sparse_steps"] += int(use_sparse)
        else:
            fset.probe(keys_batch, out=hits_bufs[buf], stream=lane_sh[buf], gated=gated)

    def step_set():
        set_step(claim())

    region = {}  # HIP events on the kernels' stream around the last timed region

    def timed(fn, k, lanes=None):
        with guard("timed"):
            return _timed(fn, k, lanes)

    def _timed(fn, k, lanes=None):
        lanes = lane_streams if lanes is None else lanes
        torch.cuda.synchronize(dev)  # all streams: every exchange of the K steps is inside
        if use_dist:
            dist.barrier()
            torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        # every stream is idle here, so the lanes' first steps (issued after
        # e0) cannot start before it; no cross-stream wait is issued: each
        # wait_stream costs ~9 us of host time, which at K = 20 delays the
        # first step (and every step after it) by ~19 us
        e0.record(stream)
        for _ in range(k):
            fn()
        for st in lanes[1:]:
            stream.wait_stream(st)  # e1 after every lane's last step
        e1.record(stream)
        torch.cuda.synchronize(dev)
        if use_dist:
            dist.barrier()
        el = time.perf_counter() - t0
        region["ms"], region["k"] = e0.elapsed_time(e1), k
        if use_dist:
            t = torch.tensor([el], dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # secondary legs time LK steps: a sub-0.1 ms step timed 20 times is mostly
    # the region's fill and drain (the headline leg keeps exactly --steps)
    LK = max(args.steps, args.leg_steps)
    probes_per_step = n * nf_total
    legs = {}
    for name, fn in (("tiled", step_tiled), ("filterset", step_set)):
        with guard("warmup"):
            for _ in range(args.warmup):
                fn()
            torch.cuda.synchronize(dev)
        el_leg = timed(fn, args.steps)
        legs[name] = {"el": el_leg, "value": probes_per_step / (el_leg / args.steps),
                      "ms_per_step": el_leg / args.steps * 1e3, "fn": fn,
                      "region_us_per_step": region["ms"] * 1e3 / region["k"]}
    best = max(legs, key=lambda k: legs[k]["value"])
    el = legs[best]["el"]
    step = legs[best]["fn"]
    ms_step = el / args.steps * 1e3
    value = legs[best]["value"]

    # ---- separate profiled pass: per-kernel durations from HIP events on `sh`
    def kernel_ms(names, fn, k):
        L.cb_profile_reset()
        L.cb_profile_enable(1)
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        L.cb_profile_enable(0)
        out = {}
        for nm in names:
            tot = __import__("ctypes").c_double()
            cnt = __import__("ctypes").c_uint64()
            L.cb_profile_read(nm.encode(), __import__("ctypes").byref(tot), __import__("ctypes").byref(cnt))
            if cnt.value:
                out[nm] = {"avg_us": tot.value * 1e3 / cnt.value, "launches": int(cnt.value)}
        return out

    def cold_run(names, fn, reps=8, clean=False):
        def reset():
            step_no[0] = 0  # the rep's step runs on lane 0 (= `stream`, where the events are)
        return _cold_steps(torch, dist, use_dist, dev, stream, L, names, fn, reset, reps, clean)

    probe_kernels = ["k_part_probe", "k_tile_probe", "k_masks_to_hits", "k_probe_direct",
                     "k_set_probe"]
    kprof = kernel_ms(probe_kernels, step, args.steps)
    cold = None
    if not args.no_cold:
        cold_ms, cold_k = cold_run(probe_kernels, step)
        cold = {"value": round(probes_per_step / (cold_ms * 1e-3), 1), "ms_per_step": round(cold_ms, 4),
                "kernels_us": cold_k, "protocol": "1 GiB device write before each of 8 reps, median"}
        clean_ms, clean_k = cold_run(probe_kernels, step, clean=True)
        cold["clean_caches"] = {"value": round(probes_per_step / (clean_ms * 1e-3), 1),
                                "ms_per_step": round(clean_ms, 4), "kernels_us": clean_k,
                                "protocol": "the same write, then a 512 MiB read, before each rep"}

    # rotating batches: 4 different lookup batches over the same filters, one
    # per step in turn, so a step cannot find the set lines of its own
    # previous run in the Infinity Cache (warm = the same batch every step)
    rot = None
    if best == "filterset":
        nrot = 4
        shift = (n // 2 // nf_total) or 1
        rot_keys = [keys_batch] + [
            lsmt_amd.DeviceKeys(torch.from_numpy(workload.probe_lookups(
                n, nf_total, kpf, seed_base=seed_base, absent_seed=absent_seed + 7919 * r,
                shift=r * shift)).to(dev)) for r in range(1, nrot)]
        rot_i = [0]

        def step_rot():
            buf = claim()
            fset.probe(rot_keys[rot_i[0] % nrot], out=hits_bufs[buf], stream=lane_sh[buf])
            rot_i[0] += 1
            exchange(buf)

        for _ in range(args.warmup):
            step_rot()
        rel = timed(step_rot, LK)
        rprof = kernel_ms(probe_kernels, step_rot, LK)
        rot = {"value": round(probes_per_step / (rel / LK), 1),
               "ms_per_step": round(rel / LK * 1e3, 4), "steps": LK,
               "kernels_us": {k: round(v["avg_us"], 2) for k, v in rprof.items()},
               "batches": nrot}
        del rot_keys
    kprof_alt = kernel_ms(probe_kernels, legs["tiled" if best == "filterset" else "filterset"]["fn"], args.steps)
    dominant = max(kprof, key=lambda k: kprof[k]["avg_us"]) if kprof else None

    if best == "tiled":
        # algorithmic bytes per probe launch:
        # F*m/8*tau (each filter streamed once) + 16*n (keys) + F*n/8 (hit bitmaps)
        tau = 1.0 - np.exp(-n * 1.0155 / (m / 512.0))
        alg_bytes = F * m / 8 * tau + 16 * n + F * n / 8
        alg_def = "F*m/8*tau + 16n + F*n/8 (SURVEY.md §8d C3 row)"
    else:
        # bit-sliced layout (SURVEY.md §8d "alternative layout"): 64 B x distinct
        # sectors touched by the a/b word reads + 16 B/key + the hit bitmaps
        sectors, rand_reads = _set_sectors(filters, look_np, m, F)
        alg_bytes = 64 * sectors + 16 * n + F * n / 8
        alg_def = f"64 B x {sectors} distinct sectors + 16n + F*n/8 (SURVEY.md §8d alternative layout)"
    # the same FilterSet step on ONE lane (every launch on `stream`, none
    # overlapping): the kernel's own back-to-back duration, so the roofline
    # does not depend on the lane count (roofline.frac_one_lane)
    one_lane_us = None
    if best == "filterset" and not use_dist:
        def step_one():
            fset.probe(keys_batch, out=hits_bufs[0], stream=sh)

        for _ in range(args.warmup):
            step_one()
        timed(step_one, LK)
        one_lane_us = region["ms"] * 1e3 / region["k"]

    roof = None
    if dominant:
        # Kernel duration for the roofline: HIP events recorded on the kernels'
        # stream around the K timed steps, divided by K. Without an exchange
        # the FilterSet step is exactly one k_set_probe launch, so this is the
        # kernel's back-to-back average and can never exceed the step time
        # (per-launch cb_profile events add their own gaps; kept as kernels_us).
        one_kernel = best == "filterset" and not use_dist
        kus = legs[best]["region_us_per_step"] if one_kernel else \
            min(kprof[dominant]["avg_us"], legs[best]["ms_per_step"] * 1e3)
        kus_src = (("HIP events around the timed region / K (one launch per step; " +
                    (f"launches overlap {P} deep on {P} lanes, so this is each launch's share of the chip "
                     f"and kernel_avg_us_per_launch_events is one launch's own duration)" if P > 1 else
                     "one lane)")) if one_kernel else "cb_profile per-launch HIP events, capped at the step time")
        dur_s = kus * 1e-6
        ach = alg_bytes / dur_s / 1e9
        # PMC bytes are recorded for the default C3 shape only (profiles/pmc_*.json)
        c3_default = (args.workload == "c3" and n == 1 << 20 and F == 32 and m == 1 << 26 and kpf == 1 << 19)
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": _pmc_traffic(dominant) if c3_default else None,
                "kernel": dominant, "kernel_avg_us": round(kus, 2), "kernel_avg_source": kus_src,
                "kernel_avg_us_per_launch_events": round(kprof[dominant]["avg_us"], 2),
                "algorithmic_bytes": int(alg_bytes), "algorithmic_def": alg_def,
                "step_effective_GBps": round(alg_bytes / (el / args.steps) / 1e9, 1)}
        if one_lane_us:
            roof["kernel_avg_us_one_lane"] = round(one_lane_us, 2)
            roof["frac_one_lane"] = round(alg_bytes / (one_lane_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
        if c3_default:
            roof["traffic_source"] = _pmc_source("c3")
            roof["profile_check"] = _profile_check("c3", [dominant], alg_bytes, roof.get("frac_one_lane"))
        if roof["traffic"]:  # the memory-side bytes the kernel moves (PMC), at the same time per launch
            roof["traffic_GBps"] = round(roof["traffic"] / dur_s / 1e9, 1)
            roof["traffic_frac"] = round(roof["traffic"] / dur_s / 1e9 / HBM_PEAK_GBS, 4)
            roof["traffic_note"] = ("every random 4-B set read fills a whole 128-B L2 line (PMC: TCC_EA0_RDREQ_128B), "
                                    "so the fabric moves ~2.2x the algorithmic bytes; hipDeviceMallocUncached "
                                    "memory and non-temporal loads fetch the same (profiles/ubench_random_r01.json)")
        if best == "filterset":
            rr = _random_read_roofline()
            if rr:
                got = rand_reads / dur_s
                roof["random_read_roofline"] = {
                    "reads_per_launch": rand_reads, "achieved_reads_per_s": round(got, 1),
                    "peak_reads_per_s": rr, "frac": round(got / rr, 4),
                    "source": "profiles/ubench_random_r01.json (256 MiB table, hipMalloc)"}
                if one_lane_us:
                    roof["random_read_roofline"]["frac_one_lane"] = round(rand_reads / (one_lane_us * 1e-6) / rr, 4)

    # maintenance cost of the set on the flush path: one new filter into an
    # empty slot (sparse OR of its set bits)
    fset2 = lsmt_amd.FilterSet(m, width=32, device=local)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    fset2.assign(0, filters[0], stream=sh)
    torch.cuda.synchronize(dev)
    set_assign_ms = (time.perf_counter() - t0) * 1e3
    del fset2

    # ---- zone-map gate: each slot's ZoneMap built on the
    # device from its table's keys (the zone_map.update loop of SsTable::create),
    # then the same probe with SsTable::get's full gate (src/sstable.rs:138).
    zone = None
    if not args.no_zone:
        zkeys = [torch.from_numpy(workload.key_range(seed_base + f, kpf)).to(dev) for f in range(f_lo, f_lo + F)]
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i, zk in enumerate(zkeys):
            fset.zone_from_keys(i, lsmt_amd.DeviceKeys(zk), stream=sh)
        torch.cuda.synchronize(dev)
        zone_build_s = time.perf_counter() - t0
        del zkeys

        def step_gated():
            set_step(claim(), gated=True)

        for _ in range(args.warmup):
            step_gated()
        gel = timed(step_gated, LK)
        gprof = kernel_ms(["k_set_probe_gated"], step_gated, LK)
        gated_hits = int(np.unpackbits(hits_bufs[(step_no[0] - 1) % P].cpu().numpy().view(np.uint8)).sum())
        zone = {"value": round(probes_per_step / (gel / LK), 1), "unit": "gated probes/s",
                "ms_per_step": round(gel / LK * 1e3, 4), "steps": LK,
                "kernels_us": {k: round(v["avg_us"], 2) for k, v in gprof.items()},
                "zone_build_keys_per_s": round(F * kpf / zone_build_s, 1),
                "gated_hits_last_step": gated_hits,
                "note": "C3 tables hold random keys, so every zone spans ~the whole key space: "
                        "this measures the gate's cost; 'partitioned' measures it where it rejects"}

    # ---- the zone gate where it rejects: range-partitioned tables (an L1-L4
    # style level, each table holding a contiguous key range), so exactly one
    # zone contains any key and the gate clears every Bloom false positive
    # of the other tables (src/sstable.rs:138, src/zonemap.rs:37-42)
    if not args.no_zone and rank == 0 and world == 1:
        zone["partitioned"] = zone_partitioned_leg(args, torch, dev, local, sh, F, m, kpf, n, timed, kernel_ms,
                                                   probes_per_step, lsmt_amd, workload)

    # ---- read path: the C3 tables as real SSTable data
    # files in HBM; one step = gated probe + Database::get's newest-first walk
    # (binary search of the candidates, base64 decode of the found values)
    read = None
    if not args.no_read and not args.no_zone:
        t0 = time.perf_counter()
        files = [torch.from_numpy(workload.sstable_bytes(k, workload.table_value(k, f)))
                 for f, k in ((f, workload.key_range(seed_base + f, kpf)) for f in range(f_lo, f_lo + F))]
        gen_s = time.perf_counter() - t0
        dfiles = [f.to(dev) for f in files]
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        tables = [lsmt_amd.Table(f, device=local, stream=sh) for f in dfiles]
        torch.cuda.synchronize(dev)
        index_s = time.perf_counter() - t0
        file_bytes = sum(int(f.numel()) for f in files)
        del files
        newest_first = tables[::-1]  # Database::get: tables.iter().rev()
        rows = np.arange(F)[::-1].copy()
        # one batch per step, batches alternating over the lanes (as the probe
        # legs): each lane has its own gate rows and outputs, and get_many
        # only enqueues (total read from val_off[n] afterwards), so one
        # batch's search overlaps the next batch's gated probe
        which_l = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(P)]
        voff_l = [torch.empty(n + 1, dtype=torch.int64, device=dev) for _ in range(P)]
        vals_l = [torch.empty(n * 16, dtype=torch.uint8, device=dev) for _ in range(P)]
        hits_l = [torch.empty((F, words), dtype=torch.int64, device=dev) for _ in range(P)]

        def step_read():
            b = claim()
            fset.probe(keys_batch, out=hits_l[b], stream=lane_sh[b], gated=True)
            lsmt_amd.get_many(newest_first, keys_batch, hits=hits_l[b], hit_rows=rows,
                              out=(which_l[b], voff_l[b], vals_l[b]), stream=lane_sh[b], wait=False)

        def step_fused():
            """Database::get in one launch (cb_set_get_many_fixed): the same
            zone + Bloom gate computed from the FilterSet inside the search
            kernel, so no gate rows are written or read."""
            b = claim()
            lsmt_amd.get_many(newest_first, keys_batch, filterset=fset, hit_rows=rows,
                              out=(which_l[b], voff_l[b], vals_l[b]), stream=lane_sh[b], wait=False)

        rforms = {}
        for name, fn, kn in (("two_step", step_read, ["k_set_probe_gated", "k_get_many", "k_tile_scan", "k_b64_decode"]),
                             ("fused", step_fused, ["k_set_get_many", "k_tile_scan", "k_b64_decode"])):
            for _ in range(args.warmup):
                fn()
            el_r = timed(fn, LK)
            rprof = kernel_ms(kn, fn, LK)
            torch.cuda.synchronize(dev)
            rforms[name] = {"value": round(n / (el_r / LK), 1), "ms_per_step": round(el_r / LK * 1e3, 4), "steps": LK,
                            "kernels_us": {k: round(v["avg_us"], 2) for k, v in rprof.items()},
                            "which": which_l[0].clone(), "voff": voff_l[0].clone()}
            assert all(torch.equal(which_l[0], w) and torch.equal(voff_l[0], v) for w, v in zip(which_l, voff_l))
        same = (torch.equal(rforms["fused"]["which"], rforms["two_step"]["which"]) and
                torch.equal(rforms["fused"]["voff"], rforms["two_step"]["voff"]))
        for f in rforms.values():
            del f["which"], f["voff"]
        rbest = max(rforms, key=lambda k: rforms[k]["value"])
        found = int((which_l[0] >= 0).sum().item())
        got = [int(voff_l[0][n].item())]
        read = {"metric": "gets/s: 1M keys through zone+Bloom gate, binary search and base64 decode over "
                          f"{F} SSTable data files ({kpf} lines each) in HBM",
                "value": rforms[rbest]["value"], "unit": "keys/s", "form": rbest,
                "ms_per_step": rforms[rbest]["ms_per_step"], "kernels_us": rforms[rbest]["kernels_us"],
                "forms": rforms, "fused_equals_two_step": bool(same),
                "found": found, "value_bytes": got[0], "pipeline_lanes": P,
                "files_bytes": file_bytes, "index_build_GBps": round(file_bytes / index_s / 1e9, 2),
                "file_generation_s": round(gen_s, 2)}
        if rank == 0 and world == 1 and not args.no_cpu:
            from oracle import oracle
            sample = 1 << 15
            ot = [oracle.OracleTable(workload.sstable_bytes(k, workload.table_value(k, f)))
                  for f, k in ((f, workload.key_range(seed_base + f, kpf)) for f in range(f_lo, f_lo + F))][::-1]
            hs = hits_l[0].cpu().numpy().view(np.uint64)[rows]
            hs = np.ascontiguousarray(hs[:, : sample // 64])
            t0 = time.perf_counter()
            ow, ovoff, ovals = oracle.get_many(ot, hs, np.ascontiguousarray(look_np[:sample].reshape(-1)),
                                               np.arange(0, 16 * (sample + 1), 16, dtype=np.uint64))
            read["cpu_baseline"] = {"value": round(sample / (time.perf_counter() - t0), 1), "unit": "keys/s",
                                    "cores": 1, "kind": "port",
                                    "sample": f"oracle get_many over the first {sample} keys with the same gate bits"}
            # the same sample checked (lanes hold the fused form's answers, the
            # leg that ran last): table index, value offsets and value bytes
            gvo = voff_l[0][: sample + 1].cpu().numpy().astype(np.uint64)
            read["oracle_sample_bit_exact"] = bool(
                np.array_equal(which_l[0][:sample].cpu().numpy(), ow) and np.array_equal(gvo, ovoff) and
                bytes(vals_l[0][: int(gvo[-1])].cpu().numpy()) == ovals)
            del ot
        del tables, dfiles
    if zone is not None:
        fset.assign_all(filters, stream=sh)  # zones reset; the set is unchanged otherwise

    # ---- the reference's own read shape: 300 auto-flushed tables (1024
    # entries each, m = 1024, src/lib.rs:72,105, src/sstable.rs:44,59) in
    # one wide FilterSet, Database::get over all of them in one launch
    wide = None
    if not args.no_wide and rank == 0 and world == 1:
        wide = wide_fanout_leg(args, torch, dev, local, lane_streams, LK, timed, kernel_ms, lsmt_amd, workload)
        log(f"[wide] {wide['value'] / 1e6:.1f} M gets/s over {wide['tables']} tables, "
            f"oracle {wide.get('oracle_sample_bit_exact')}")

    # ---- flush producer: SsTable::create on the device
    # for a 1M-entry memtable (16-B keys, 16-B insert_ts values): data file +
    # line index + Bloom filter (m = 2^26) + zone bounds, inputs in HBM
    flush = None
    if not args.no_flush:
        nf_e = args.flush_entries
        fk = workload.key_range(7000, nf_e)
        fv = workload.table_value(fk, 1)
        res = {}

        def shared_prefix_keys(n, seed):
            # every key under one 8-byte prefix ("default:" + 8 hex digits of a
            # permutation): one bin for the bin sort, so the merge sort it
            # enqueues after itself runs (capi_sstable.cpp sstable_enqueue)
            perm = np.random.default_rng(seed).permutation(n).astype(np.uint32)
            hexd = np.frombuffer(b"0123456789abcdef", np.uint8)
            out = np.empty((n, 16), np.uint8)
            out[:, :8] = np.frombuffer(b"default:", np.uint8)
            for c in range(8):
                out[:, 8 + c] = hexd[(perm >> (28 - 4 * c)) & 15]
            return out

        for label, keys_np in (("sorted", workload.sort_keys16(fk)), ("unsorted", fk),
                               ("unsorted_shared_prefix", shared_prefix_keys(nf_e, 7001))):
            kd = torch.from_numpy(np.ascontiguousarray(keys_np.reshape(-1))).to(dev)
            vd = torch.from_numpy(np.ascontiguousarray(fv.reshape(-1))).to(dev)
            ko = torch.from_numpy(np.arange(0, 16 * (nf_e + 1), 16, dtype=np.int64)).to(dev)
            kbatch = lsmt_amd.KeyBatch(n=nf_e, data=kd, offsets=ko)
            vbatch = lsmt_amd.KeyBatch(n=nf_e, data=vd, offsets=ko)
            made = []
            fl_no = [0]

            def step_flush(lanes_n=P):
                # enqueue-only (cb_sstable_create_bounded): the table finalises
                # on first use; tables are kept, as an LSM keeps its SSTables.
                # Consecutive flushes alternate over the pipeline lanes (as
                # the probe and read legs), each lane with its own stream and
                # workspace
                i = fl_no[0] % lanes_n
                fl_no[0] += 1
                made.append(lsmt_amd.sstable_create((kbatch, vbatch), m=1 << 26, device=local, stream=lane_sh[i],
                                                    wait=False))

            k_fl = max(3, LK // 4)
            # warm-up: as many flushes as the timed region, then freed, so the
            # timed region's allocations come from the library's block pool
            # (not --warmup flushes: they are all held until the warm-up ends,
            # ~60 MB of HBM each, and 3000 of them exhausted the device)
            for _ in range(max(1, k_fl)):
                step_flush()
            for t, _, _ in made:
                t.wait()
            made.clear()
            fel = timed(step_flush, k_fl)
            for t, _, _ in made:
                t.wait()  # finalised after the region (host reads of the results only)
            made.clear()
            # one flush at a time (one stream): the latency one flush pays
            fel1 = timed(lambda: step_flush(1), k_fl, lanes=lane_streams[:1])
            for t, _, _ in made:
                t.wait()
            last = made[-1]
            made.clear()
            made.append(last)
            fprof = kernel_ms(["k_sorted_check", "k_entry_sort", "k_bin_count", "k_bin_offsets", "k_bin_scatter", "k_bin_sort", "k_tile_scan",
                               "k_format", "k_line_count", "k_line_emit", "k_line_finish", "k_line_keys",
                               "k_build_part", "k_build_tile", "k_insert_direct"], step_flush, min(k_fl, 20))
            for t, _, _ in made:
                t.wait()
            out_bytes = last[0].nbytes
            if label == "unsorted" and rank == 0 and world == 1 and not args.no_cpu:
                flush_file = last[0].data()  # checked against the oracle below
            res[label] = {"entries_per_s": round(nf_e / (fel / k_fl), 1), "ms_per_flush": round(fel / k_fl * 1e3, 3),
                          "flushes": k_fl, "pipeline_lanes": P,
                          "form": "enqueue-only creates (tables finalised after the region)",
                          "one_lane": {"ms_per_flush": round(fel1 / k_fl * 1e3, 3),
                                       "entries_per_s": round(nf_e / (fel1 / k_fl), 1)},
                          "file_bytes": out_bytes, "file_GBps": round(out_bytes / (fel / k_fl) / 1e9, 2),
                          "kernels_us": {k: round(v["avg_us"], 2) for k, v in fprof.items()}}
            del made, kd, vd, ko
        flush = {"metric": f"SsTable::create entries/s ({nf_e} entries, 16-B keys, 16-B values, m=2^26), "
                           "data file + index + Bloom filter + zone, inputs in HBM",
                 "kernels_us_source": "library HIP events around each launch (cb_profile): a launch's figure also "
                                      "holds its dispatch gap; rocprofv3 durations are in profiles/ (DESIGN.md §6)",
                 "sorted_input": res["sorted"], "unsorted_input": res["unsorted"],
                 "unsorted_shared_prefix_input": res["unsorted_shared_prefix"]}
        if rank == 0 and world == 1 and not args.no_cpu:
            from oracle import oracle
            sample = 1 << 17
            ents = [(bytes(fk[i]), bytes(fv[i])) for i in range(sample)]
            t0 = time.perf_counter()
            oracle.sstable_create(ents)
            flush["cpu_baseline"] = {"value": round(sample / (time.perf_counter() - t0), 1), "unit": "entries/s",
                                     "cores": 1, "kind": "port",
                                     "sample": f"oracle sstable_create on {sample} unsorted entries (file only)"}
            # the timed unsorted flush's whole file against the oracle's stable sort + format
            ents = [(bytes(fk[i]), bytes(fv[i])) for i in range(nf_e)]
            flush["oracle_file_bit_exact"] = bool(oracle.sstable_create(ents) == flush_file)
            del ents, flush_file

    # ---- C2 build: 1M keys -> one fresh 16 MiB filter (zero-fill + batched
    # insert): c2_leg, also run alone by `--leg c2` (tools/profile_round.sh c2)
    build = c2_leg(args, torch, dist, dev, local, world, use_dist, red_dev, LK, args.warmup,
                   _LANES[:args.build_streams], cold=not args.no_cold)

    # ---- PCIe-inclusive end-to-end probe (pinned host keys -> host hits)
    e2e = None
    if not args.no_e2e and rank == 0:
        # keys arrive in pinned host memory from the query layer and the hit
        # bitmap returns there (SURVEY.md §8d end-to-end leg): the FilterSet
        # probe reading keys / writing hits over PCIe from the kernel
        # (zero-copy), and the per-filter probe with one staged H2D and one D2H
        look_pin = torch.from_numpy(look_np).pin_memory()
        hits_host = torch.zeros((F, words), dtype=torch.int64).pin_memory()
        hb = lsmt_amd.KeyBatch(n=n, key_len=16, keys=look_pin)

        def wall(fn, k):
            fn()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(k):
                fn()
            return (time.perf_counter() - t0) / k

        k_e2e = max(5, args.steps // 2)
        t_set = wall(lambda: fset.probe(hb, out=hits_host, stream=sh), k_e2e)
        pipelined = int(L.cb_last_path()) == 4
        t_tiled = wall(lambda: lsmt_amd.probe(filters, hb, out=hits_host, stream=sh), k_e2e)
        # the same FilterSet probe with pinned hipMemcpyAsync H2D / D2H around it
        look_dev = torch.empty_like(look)
        hits_dev = torch.empty((F, words), dtype=torch.int64, device=dev)
        db = lsmt_amd.KeyBatch(n=n, key_len=16, keys=look_dev)

        def staged():
            look_dev.copy_(look_pin, non_blocking=True)
            fset.probe(db, out=hits_dev, stream=sh)
            hits_host.copy_(hits_dev, non_blocking=True)
            torch.cuda.synchronize(dev)

        t_staged = wall(staged, k_e2e)
        e2e = {"probes_per_s": round(n * F / t_set, 1), "ms_per_step": round(t_set * 1e3, 3),
               "path": "filterset" + (", zero-copy (kernel loads keys / stores hits over PCIe)" if pipelined else ""),
               "h2d_bytes": 16 * n, "d2h_bytes": F * words * 8, "host_buffers": "pinned",
               "pcie_GBps": round((16 * n + F * words * 8) / t_set / 1e9, 1),
               "alt_filterset_staged": {"probes_per_s": round(n * F / t_staged, 1),
                                        "ms_per_step": round(t_staged * 1e3, 3),
                                        "form": "pinned hipMemcpyAsync H2D, set probe, D2H, one stream"},
               "alt_per_filter_tiled": {"probes_per_s": round(n * F / t_tiled, 1),
                                        "ms_per_step": round(t_tiled * 1e3, 3)}}

    # ---- the per-key drop-in call (SsTable::get's bloom.may_contain(key),
    # src/sstable.rs:138): one host thread through the C ABI, host mirror vs
    # one-key GPU probe, at the product's m = 1024 and the C3 filter size
    may_contain = None
    if rank == 0 and world == 1:
        may_contain = may_contain_latency()

    # ---- BASELINE C4 and C5 in the same line (HIP-event timed, roofline,
    # golden + oracle checks): C4's 64 builds split over the ranks (strong
    # scaling); C5's per-GPU slice (rank r: filters 32(r mod 8) .. +31 of 256)
    c4 = c5 = None

    def run_c5():
        c5 = c5_leg(args, torch, dev, local, world, rank, max(args.steps, LK // 4), args.warmup,
                    args.probe_streams, True, red_dev, dist, use_dist)
        log(f"[c5] {c5['value'] / 1e12:.3f} T probes/s, {c5['region_us_per_step']} us/step, "
            f"frac {c5['roofline']['frac']}, golden {c5.get('golden_slice_bit_exact')}")
        return c5

    if args.workload == "c3" and not args.no_c4:
        c4 = c4_leg(args, torch, dist, world, rank, local, dev, use_dist, red_dev, LK, args.warmup,
                    args.probe_streams, check=True, oracle_sample=0 if args.no_cpu else 4)
        c4["roofline"] = c4_roofline(c4, world)
        if rank == 0 and world == 1 and not args.no_cpu:
            c4["cpu_baseline"] = c4_cpu_baseline(64, 1 << 18, 1 << 25)
        log(f"[c4] {c4['value'] / 1e9:.1f} G keys/s, {c4['region_us_per_step']} us/step, "
            f"frac {c4['roofline']['frac']}, golden {c4.get('golden_all_filters_bit_exact')}")
    if args.workload == "c3" and not args.no_c5:
        c5 = run_c5()

    if args.check:
        # Every rank checks its own rows and, in the exchanged map, the rows
        # of the next rank, so each rank's slice is verified as received by
        # another rank; the verdicts are combined over all ranks.
        from oracle import oracle

        def oracle_rows(lo, hi):
            refs = []
            for f in range(lo, hi):
                o = oracle.OracleFilter(m)
                o.insert_fixed(workload.key_range(seed_base + f, kpf))
                refs.append(o)
            return oracle.probe_fixed(refs, look_np, threads=8)

        step()  # the headline leg again (the zone leg ran after it)
        torch.cuda.synchronize(dev)
        expect = oracle_rows(f_lo, f_lo + F)
        got = hits_bufs[(step_no[0] - 1) % P].cpu().numpy().view(np.uint64)
        good = bool(np.array_equal(got, expect))
        if use_dist:
            full = hits_all_bufs[(step_no[0] - 1) % P].cpu().numpy().view(np.uint64)
            good &= bool(np.array_equal(full[f_lo:f_lo + F], expect))
            if world > 1:
                nlo, nhi = shard_range(nf_total, world, (rank + 1) % world)
                good &= bool(np.array_equal(full[nlo:nhi], oracle_rows(nlo, nhi)))
            flag = torch.tensor([1 if good else 0], dtype=torch.int32, device=red_dev)
            with guard("check"):
                dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            good = bool(flag.item())
        assert good, "bench hits differ from the oracle"
        if rank == 0:
            log("[check] hits bit-exact vs oracle" +
                (" (local rows on every rank, and every rank's rows in another rank's exchanged map)"
                 if use_dist else ""))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.workload == "c3":
        cpu = cpu_baseline(look_np, F, m, kpf, args.build_keys, args.build_m_bits)
        log(f"[cpu] {cpu}")

    x_fit = None
    if use_sparse:  # every step's packs held all set bits: every exchanged map was complete
        x_fit = bool(int(x_ok.item()))
        if not x_fit:
            log(f"[rank {rank}] ERROR: a sparse exchange overflowed cap={cap}; its map was incomplete, "
                "so the timed steps did not all exchange the full map: the line is marked invalid")

    # the BASELINE config name only when the shape is exactly that config's
    c3_shape = (n == 1 << 20 and F == 32 and m == 1 << 26 and kpf == 1 << 19)
    c5_shape = (n == 10_000_000 and F == 32 and m == 1 << 26 and kpf == 1 << 19 and seed_base == 1000)
    wl_label = ("C3" if args.workload == "c3" and c3_shape else
                "C5 rank-slice" if args.workload == "c5" and c5_shape else "custom")
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "probes/s",
            "n_gpus": xcomm.world if xcomm is not None else world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (splitmix64 hex keys, SURVEY.md §8d)",
            "config": {"workload": f"{wl_label} probe: {n} 16-B keys x {F} filters/GPU x {m // 8 // 2**20} MiB "
                                   f"(m=2^{m.bit_length() - 1}), filters built from {kpf} keys each",
                       "n_keys": n, "filters_per_gpu": F, "filters_total": nf_total, "m_bits": m,
                       "keys_per_filter": kpf,
                       "parallelism": "filter-sharded" + (
                           (", RCCL all-gather of hit bitmaps" + (
                               " as set-bit positions (sparse packs)" if use_sparse else
                               " after each probe"))
                           if use_dist else ""),
                       "pipeline_lanes": P},
            "exchange": (dict(xstats, mode="sparse", cap=cap, all_fit=x_fit) if use_sparse else
                         {"mode": "dense"} if use_dist else None),
            "path": best,
            "kernels_us": {k: round(v["avg_us"], 2) for k, v in kprof.items()},
            "alt_paths": {k: {"value": round(v["value"], 1), "ms_per_step": round(v["ms_per_step"], 4)}
                          for k, v in legs.items() if k != best},
            "alt_kernels_us": {k: round(v["avg_us"], 2) for k, v in kprof_alt.items()},
            "filterset": {"build_all_ms": round(set_build_ms, 3), "assign_one_empty_slot_ms": round(set_assign_ms, 3),
                          "bytes": m * (4 if F <= 32 else 8)},
            "cold": cold, "rotating_batches": rot, "roofline": roof, "cpu_baseline": cpu, "build": build, "e2e": e2e,
            "zone_gate": zone, "read_path": read, "flush": flush, "may_contain": may_contain,
            "c4": c4, "c5": c5, "wide_fanout": wide,
        }
        if rccl_world is not None:
            line["rccl_world"] = rccl_world
        if x_fit is False:
            line["valid"] = False
        if rehearse:
            line["rehearsal"] = (f"{world} ranks on ONE GPU over the host transport (gloo): checks the N-rank "
                                 "flow, not a scaling measurement")
            line["valid"] = False
        emit(line, result, args.full_line)
    if use_dist:
        with guard("teardown"):
            torch.cuda.synchronize(dev)
            dist.barrier()
        if _WD is not None:
            _WD.comm = None
        xcomm.close()
        dist.destroy_process_group()
    if x_fit is False:
        sys.exit(3)


# ---- the result line -------------------------------------------------------
# The driver keeps ~9 KB of a run's stdout, and round 5's 14.7 KB line lost
# its first legs (build, e2e, cold) to it. Stdout therefore carries a compact
# line: the prose fields (what each number means, its sources; DESIGN.md §6
# "Bench line fields" keeps them) and per-kernel breakdowns of the secondary
# legs go, floats are rounded, and the keys are ordered so that the legs the
# driver's tail must show (build, e2e, cold, may_contain) come last. The full
# line goes to --full-line PATH when asked.
LINE_BUDGET = 8000
PROSE = {"note", "kernels_us_source", "kernel_avg_source", "algorithmic_def", "traffic_note", "host_issued_note",
         "protocol", "form", "oracle_sample", "launches_per_batch", "sink", "cpus", "slice", "source", "kernels",
         "metric", "sample", "path", "tables", "forms", "cpu_model"}
# per-leg keys dropped from the compact line (kept in the full line)
DETAIL = {"flush": {"kernels_us", "file_bytes", "flushes", "pipeline_lanes"},
          "read_path": {"files_bytes", "file_generation_s", "value_bytes", "pipeline_lanes"},
          "may_contain": {"m_bits", "keys", "probe_keys", "hits", "mirror_calls", "gpu_calls", "sink"},
          "zone_gate": {"gated_hits_last_step", "zone_build_keys_per_s", "bloom_pass_pairs", "gate_pass_pairs"},
          "profile_check": {"traced_run_events_us", "plain_run_events_us", "ratio_to_traced_run_events"},
          "c4": {"filters_total", "keys_per_filter", "m_bits", "warmup", "pipeline_lanes", "lanes_region_us_per_step"},
          "c5": {"n_keys", "filters", "m_bits", "pipeline_lanes"},
          "wide_fanout": {"set_width", "lookups", "table_build_s"},
          "e2e": {"h2d_bytes", "d2h_bytes", "host_buffers"},
          "random_read_roofline": {"reads_per_launch", "achieved_reads_per_s", "peak_reads_per_s"}}
TAIL = ("build", "e2e", "cold", "may_contain")  # last in the line: what the driver's tail must hold
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _compact(v, key=None, top=False, leg=None):
    """v without its prose and detail fields (DETAIL applies at every depth
    of its leg, and to dicts of its own name), floats rounded."""
    if isinstance(v, dict):
        out = {}
        drop = DETAIL.get(key, set()) | DETAIL.get(leg, set())
        for k, x in v.items():
            if k in drop:
                continue
            if k in PROSE and isinstance(x, (str, list, dict)) and not top and not (
                    key == "cpu_baseline" and k in ("sample", "cpu_model")):
                continue
            if k == "kernels_us" and isinstance(x, dict):  # {kernel: {avg_us, launches}} -> {kernel: avg_us}
                x = {kk: (vv["avg_us"] if isinstance(vv, dict) else vv) for kk, vv in x.items()}
            out[k] = _compact(x, k, leg=k if top else leg)
        return out
    if isinstance(v, list):
        return [_compact(x, key, leg=leg) for x in v]
    if isinstance(v, float):
        return int(round(v)) if abs(v) >= 1000 else round(v, 4)
    return v


def compact_line(line: dict) -> dict:
    """The stdout form of the result line (see LINE_BUDGET above)."""
    c = _compact(line, top=True)
    order = [k for k in CONTRACT if k in c] + [k for k in c if k not in CONTRACT and k not in TAIL] + \
        [k for k in TAIL if k in c]
    c = {k: c[k] for k in order}
    # still over budget: the least-read secondary fields go first
    for k in ("alt_kernels_us", "rotating_batches", "filterset", "alt_paths", "kernels_us"):
        if len(json.dumps(c, separators=(",", ":"))) <= LINE_BUDGET:
            break
        c.pop(k, None)
    return c


def emit(line: dict, result, full_path=None) -> None:
    """Print the compact line to the result stream; write the full one to
    full_path when given."""
    if full_path:
        with open(full_path, "w") as fh:
            fh.write(json.dumps(line) + "\n")
    print(json.dumps(compact_line(line), separators=(",", ":")), file=result, flush=True)


def _golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as fh:
        return json.load(fh)


def _sha(a) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _timed_lanes(torch, dist, dev, use_dist, red_dev, lanes, fn, k):
    """K steps of fn between a barrier + device sync on both sides; HIP events
    on lanes[0] around them (every other lane joined into the end event).
    Returns (wall seconds, event ms), each the max over ranks."""
    with guard("timed"):
        return _timed_lanes_body(torch, dist, dev, use_dist, red_dev, lanes, fn, k)


def _timed_lanes_body(torch, dist, dev, use_dist, red_dev, lanes, fn, k):
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
        torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(lanes[0])
    for _ in range(k):
        fn()
    for st in lanes[1:]:
        lanes[0].wait_stream(st)
    e1.record(lanes[0])
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    el, ev = time.perf_counter() - t0, e0.elapsed_time(e1)
    if use_dist:
        t = torch.tensor([el, ev], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, ev = float(t[0].item()), float(t[1].item())
    return el, ev


def _all_ranks_true(torch, dist, use_dist, red_dev, ok: bool) -> bool:
    if not use_dist:
        return ok
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=red_dev)
    with guard("check"):
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())


def _kernel_us(L, torch, dev, names, fn, k):
    """Per-launch durations from the library's own HIP events (cb_profile)."""
    import ctypes
    L.cb_profile_reset()
    L.cb_profile_enable(1)
    for _ in range(k):
        fn()
    torch.cuda.synchronize(dev)
    L.cb_profile_enable(0)
    out = {}
    for nm in names:
        tot, cnt = ctypes.c_double(), ctypes.c_uint64()
        L.cb_profile_read(nm.encode(), ctypes.byref(tot), ctypes.byref(cnt))
        if cnt.value:
            out[nm] = {"avg_us": round(tot.value * 1e3 / cnt.value, 2), "launches": int(cnt.value)}
    return out


def _cold_steps(torch, dist, use_dist, dev, stream, L, names, fn, reset, reps=8, clean=False):
    """SURVEY.md §8d timing protocol, cold leg: before every rep a 1 GiB
    streaming device write evicts the L2s and the 256 MiB Infinity Cache,
    then ONE step runs (reset() first, so it runs on `stream`, where the
    events are); medians over reps of the step (HIP events on the kernels'
    stream) and of each kernel (cb_profile events). clean: a 512 MiB read
    follows the write, so the caches hold clean unrelated lines and the step
    does not also pay the write-back of the flush's dirty ones."""
    flush = torch.empty(1 << 28, dtype=torch.int32, device=dev)
    rd = torch.ones(1 << 27, dtype=torch.int32, device=dev) if clean else None
    step_ms, kus = [], {nm: [] for nm in names}
    for r in range(2 * reps):
        torch.cuda.synchronize(dev)
        if use_dist:
            with guard("cold"):
                dist.barrier()
        flush.fill_(r)
        if clean:
            rd.sum()
        reset()
        if r >= reps:
            torch.cuda.synchronize(dev)
        if r < reps:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # device-resident: the cache-evicting write (~0.2
            # ms, on the same stream) is still running while the host issues
            # the step, so the interval is the step's device time, not the
            # host's issue latency. (Round 5 first gated with a 200 us spin
            # kernel after a synchronize; the chip idles through a spin, and
            # C2 one lane measured 0.5 us slower behind an 11.7 ms one:
            # tools/c2_gate.py.)
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize(dev)
            step_ms.append(e0.elapsed_time(e1))
        else:
            for nm, v in _kernel_us(L, torch, dev, names, fn, 1).items():
                kus[nm].append(v["avg_us"])
    del flush, rd
    torch.cuda.synchronize(dev)
    # the 1.5 GiB of eviction buffers go back to the device: left in torch's
    # cache, later legs' tensors are carved from them, and the one-lane C2
    # build measured 16.5-16.6 us after the C3 cold leg against 15.4 with them
    # released (cold 22.7 -> 21.3 us; experiment r05_c2cold, HISTORY.md)
    torch.cuda.empty_cache()
    return (float(np.median(step_ms)),
            {nm: round(float(np.median(v)), 2) for nm, v in kus.items() if v})


def _gated_steps(torch, dev, fn, k, st, w=600):
    """K steps of fn queued behind W more steps of fn on st (the host issues
    faster than the device runs them, so the device starts the K timed steps
    only after the host has issued all of them): (device us per step from HIP
    events around the K, host issue us per step, whether the W steps outlasted
    the issue). The gate is real work rather than a spin kernel: behind an
    ~11.7 ms one-wave spin the same C2 builds measured 15.9-16.0 us, behind 600
    builds 15.45-15.5 (the chip idles through a spin; tools/c2_gate.py)."""
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    es = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    es.record(st)
    for _ in range(w):
        fn()
    e0.record(st)
    t1 = time.perf_counter()
    for _ in range(k):
        fn()
    t2 = time.perf_counter()
    e1.record(st)
    torch.cuda.synchronize(dev)
    # the gate's steps must still have been running when the last timed step
    # was issued
    ok = (t2 - t0) * 1e3 < es.elapsed_time(e0)
    return e0.elapsed_time(e1) * 1e3 / k, (t2 - t1) * 1e6 / k, bool(ok)


def c2_leg(args, torch, dist, dev, local, world, use_dist, red_dev, steps, warmup, lanes, cold=True):
    """BASELINE C2: one fresh 16 MiB filter (m = 2^27) built from 1M 16-B keys
    per step (clear + cb_filter_insert_fixed: SsTable::create's insert loop,
    /root/reference/src/sstable.rs:62-65, over BloomFilter::insert,
    src/bloom.rs:40-44). Consecutive steps go round-robin to len(lanes) lanes,
    each with its own filter, stream and workspace (independent flushes in
    flight); then the same build on one lane, as device time (64 builds
    queued behind 600 more) and as issued live; cold reps after a 1 GiB
    eviction. The roofline's traffic and profile check come from the C2 PMC
    summary (tools/profile_round.sh c2, one build per launch pair)."""
    import lsmt_amd
    from lsmt_amd import _lib, workload
    L = _lib.load()
    BP = len(lanes)
    b_sh = [st.cuda_stream for st in lanes]
    bk = torch.from_numpy(workload.c2_build_keys(args.build_keys)).to(dev)
    bfs = [lsmt_amd.BloomFilter(args.build_m_bits, device=local) for _ in range(BP)]
    bkb = lsmt_amd.DeviceKeys(bk)
    nstep = [0]
    nl = [BP]

    def build_step():
        i = nstep[0] % nl[0]  # (the cold reps reset nstep: they run on lane 0, where the events are)
        nstep[0] += 1
        bfs[i].clear(stream=b_sh[i])
        bfs[i].insert_batch(bkb, stream=b_sh[i])

    warm_up(torch, dev, build_step, warmup)
    el, ev_ms = _timed_lanes(torch, dist, dev, use_dist, red_dev, lanes, build_step, steps)
    region_us = ev_ms * 1e3 / steps
    # the same build on ONE lane (one flush at a time, as a real flush runs):
    # each step waits for the previous one on the stream
    nstep[0], nl[0] = 0, 1
    _, ev1_ms = _timed_lanes(torch, dist, dev, use_dist, red_dev, lanes[:1], build_step, steps)
    issued_us = ev1_ms * 1e3 / steps
    # ... and its device time: 64 steps queued behind 600 more, so the host's
    # per-step issue (Python + the C call) is not in the interval
    one_us, issue_us, gated_ok = _gated_steps(torch, dev, build_step, 64, lanes[0])
    kn = ["k_build_part", "k_build_tile", "k_insert_direct"]
    bprof = _kernel_us(L, torch, dev, kn, build_step, steps)  # one lane (nl = 1)
    if cold:
        def reset():
            nstep[0] = 0
        bcold_ms, bcold_k = _cold_steps(torch, dist, use_dist, dev, lanes[0], L, kn, build_step, reset)
        bclean_ms, bclean_k = _cold_steps(torch, dist, use_dist, dev, lanes[0], L, kn, build_step, reset, clean=True)
    nl[0] = BP
    path = int(L.cb_last_path())
    if args.check:  # every lane's filter holds the C2 bits
        from oracle import oracle
        o = oracle.OracleFilter(args.build_m_bits)
        o.insert_fixed(workload.c2_build_keys(args.build_keys))
        assert all(np.array_equal(f.bools(), o.bools()) for f in bfs), "C2 build differs from the oracle"
        del o
    del bfs, bk, bkb
    torch.cuda.synchronize(dev)
    b_alg = 16 * args.build_keys + args.build_m_bits / 8
    frac = lambda us: round(b_alg / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    kus = {k: round(v["avg_us"], 2) for k, v in bprof.items()}
    out = {"metric": "build keys/s (C2: 1M 16-B keys -> one 16 MiB filter, m=2^27)",
           "value": round(args.build_keys * world / (el / steps), 1), "unit": "keys/s",
           "ms_per_step": round(el / steps * 1e3, 4), "steps": steps, "path": path, "pipeline_lanes": BP,
           "region_us_per_step": round(region_us, 2),
           "one_lane": {"us_per_build": round(one_us, 2), "frac": frac(one_us),
                        "note": "one build at a time on one stream, device time: HIP events around 64 builds "
                                "queued behind 600 more (the latency a flush's kernels take)",
                        "queued_fully": gated_ok, "host_issue_us_per_build": round(issue_us, 2),
                        "host_issued_us_per_build": round(issued_us, 2),
                        "host_issued_note": "the same K builds issued live from Python: a build's device "
                                            "time or the host's issue time, whichever is longer"},
           "kernels_us": kus, "kernels_us_source": "library HIP events around each launch, one lane"}
    roof = {"bound": "hbm", "achieved": round(b_alg / (region_us * 1e-6) / 1e9, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": frac(region_us), "frac_one_lane": frac(one_us),
            "kernel": "k_build_part+k_build_tile", "kernel_avg_us": round(region_us, 2),
            "kernel_avg_source": f"HIP events around the timed region / K ({BP} lanes); frac_one_lane: one build "
                                 "alone, device time",
            "algorithmic_bytes": int(b_alg),
            "algorithmic_def": "16 B x 2^20 keys + 2^27/8 B (the filter written once) (SURVEY.md §8d C2 row)"}
    # PMC bytes of one build (the C2 summary holds one filter per launch pair)
    part, tile = _pmc_traffic("k_build_part", "c2"), _pmc_traffic("k_build_tile", "c2")
    c2_shape = args.build_keys == 1 << 20 and args.build_m_bits == 1 << 27
    roof["traffic"] = int(part + tile) if (part and tile and c2_shape and world == 1) else None
    if roof["traffic"]:
        roof["traffic_over_algorithmic"] = round(roof["traffic"] / b_alg, 3)
        roof["traffic_source"] = _pmc_source("c2")
    if c2_shape and world == 1:
        roof["profile_check"] = _profile_check("c2", ["k_build_part", "k_build_tile"], b_alg, roof["frac_one_lane"])
    out["roofline"] = roof
    if cold:
        out["cold"] = {"value": round(args.build_keys * world / (bcold_ms * 1e-3), 1),
                       "ms_per_step": round(bcold_ms, 4), "kernels_us": bcold_k, "frac": frac(bcold_ms * 1e3),
                       "clean_caches": {"value": round(args.build_keys * world / (bclean_ms * 1e-3), 1),
                                        "ms_per_step": round(bclean_ms, 4), "kernels_us": bclean_k,
                                        "frac": frac(bclean_ms * 1e3)}}
    return out


def c4_leg(args, torch, dist, world, rank, local, dev, use_dist, red_dev, steps, warmup, lanes_n, check, oracle_sample):
    """BASELINE C4: 64 concurrent flush builds (2^18 keys each -> m = 2^25),
    the filters split one contiguous subset per GPU (src/lib.rs:96-109,195-210:
    each flush builds its table's filter, src/sstable.rs:62-65). One step =
    clear + one batched build of this GPU's filters (cb_filter_insert_fixed_many:
    one partition and one tile launch for all of them); consecutive steps go
    round-robin to lanes_n lanes, each with its own filters and stream.
    Timed with HIP events over the region (max over ranks). check: every
    filter of every rank against the golden SHA-256s (tests/golden, made by an
    independent numpy restatement) and, for oracle_sample filters per rank,
    the C oracle's bits."""
    import lsmt_amd
    from lsmt_amd import _lib, workload
    from lsmt_amd.shard import shard_range
    L = _lib.load()
    nf_total, kpf, m = 64, 1 << 18, 1 << 25
    lo, hi = shard_range(nf_total, world, rank)
    P = lanes_n
    lanes = leg_lanes(torch, dev, P)
    keys = [torch.from_numpy(workload.c4_filter_keys(f, kpf)).to(dev) for f in range(lo, hi)]
    fsets = [[lsmt_amd.BloomFilter(m, device=local) for _ in range(lo, hi)] for _ in range(P)]
    batches = [lsmt_amd.DeviceKeys(k) for k in keys]
    nstep = [0]

    def step():
        i = nstep[0] % P
        nstep[0] += 1
        sh = lanes[i].cuda_stream
        for f in fsets[i]:
            f.clear(stream=sh)
        lsmt_amd.insert_many(fsets[i], batches, stream=sh)

    warm_up(torch, dev, step, warmup)
    el, ev_ms = _timed_lanes(torch, dist, dev, use_dist, red_dev, lanes, step, steps)
    # one lane: each batched build alone on the chip (its own duration)
    nstep[0] = 0
    P_saved, P = P, 1
    el1, ev1_ms = _timed_lanes(torch, dist, dev, use_dist, red_dev, lanes[:1], step, steps)
    # per-launch durations on ONE lane (each launch alone on the chip, so a
    # figure is that kernel's own time plus its dispatch gap, comparable with
    # rocprofv3's one-lane trace in profiles/; with three lanes a launch's
    # duration would include its overlap with the other lanes' launches)
    kus = _kernel_us(L, torch, dev, ["k_build_part", "k_build_tile"], step, min(steps, 50))
    P = P_saved
    torch.cuda.synchronize(dev)
    # the line's value is the faster schedule: at C4's size one batched build
    # fills the chip, and concurrent lanes can lose more to sharing the L2s
    # and the MALL than they gain from overlapping launch ramps (both shown)
    one = el1 < el
    el_b, ev_b = (el1, ev1_ms) if one else (el, ev_ms)
    out = {"filters_total": nf_total, "filters_this_gpu": hi - lo, "keys_per_filter": kpf, "m_bits": m,
           "steps": steps, "warmup": warmup, "pipeline_lanes": P, "lanes_used": 1 if one else P,
           "ms_per_step": round(el_b / steps * 1e3, 4),
           "region_us_per_step": round(ev_b * 1e3 / steps, 2),
           "lanes_region_us_per_step": round(ev_ms * 1e3 / steps, 2),
           "one_lane_us_per_step": round(ev1_ms * 1e3 / steps, 2),
           "value": round(nf_total * kpf / (el_b / steps), 1), "unit": "keys/s (all GPUs)",
           "kernels_us": kus, "kernels_us_source": "library HIP events around each launch, one lane"}
    if check:
        g = _golden()["c4"]
        good = True
        for i, f in enumerate(range(lo, hi)):
            for fl in fsets:
                good &= _sha(fl[i].packed().view(np.uint8)) == g["packed_sha256"][f]
        out["golden_all_filters_bit_exact"] = _all_ranks_true(torch, dist, use_dist, red_dev, good)
        if oracle_sample:
            from oracle import oracle
            picks = sorted({0, (hi - lo) // 3, 2 * (hi - lo) // 3, hi - lo - 1})[:oracle_sample]
            good = True
            for i in picks:
                o = oracle.OracleFilter(m)
                o.insert_fixed(workload.c4_filter_keys(lo + i, kpf))
                good &= all(np.array_equal(fl[i].bools(), o.bools()) for fl in fsets)
                del o
            out["oracle_sample_bit_exact"] = _all_ranks_true(torch, dist, use_dist, red_dev, good)
            out["oracle_sample"] = f"filters {[lo + i for i in picks]} of each rank vs the C oracle (byte-per-bit)"
    del fsets, keys, batches
    torch.cuda.synchronize(dev)
    return out


def c4_roofline(leg, world):
    """C4's roofline: SURVEY.md §8d's algorithmic bytes (16 B per key read +
    the filter written once) per GPU per step over the HIP-event step time;
    traffic from the committed C4 PMC summary (profiles/pmc_c4_r*.json)."""
    per_gpu = leg["filters_this_gpu"] * (16 * leg["keys_per_filter"] + leg["m_bits"] / 8)
    us = leg["region_us_per_step"]
    ach = per_gpu / (us * 1e-6) / 1e9
    r = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(ach / HBM_PEAK_GBS, 4), "kernel": "k_build_part+k_build_tile(_sub)",
         "kernel_avg_us": us, "kernel_avg_source": "HIP events around the timed region / K (the faster of the lanes and one lane: lanes_used)",
         "algorithmic_bytes": int(per_gpu),
         "algorithmic_def": "filters_this_gpu x (16 B x 2^18 keys + 2^25/8 B) (SURVEY.md §8d C4 row)",
         "frac_one_lane": round(per_gpu / (leg["one_lane_us_per_step"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
    # per step: the PMC summary is per launch of the run it was recorded on
    # (its filters_per_launch: 32 before the batch limit went to 64), so the
    # bytes scale per filter (the tile pass is k_build_tile_sub for C4's
    # batched long runs, k_build_tile otherwise)
    fpl = _pmc_field("c4", "filters_per_launch", 32)
    part = _pmc_traffic("k_build_part", "c4")
    tile = _pmc_traffic("k_build_tile_sub", "c4") or _pmc_traffic("k_build_tile", "c4")
    t = int(leg["filters_this_gpu"] * (part + tile) / fpl) if (part and tile) else None
    r["traffic"] = t if world == 1 else None
    if r["traffic"]:
        r["traffic_over_algorithmic"] = round(t / per_gpu, 3)
        r["traffic_source"] = _pmc_source("c4")
    if world == 1 and leg["filters_this_gpu"] == _pmc_field("c4", "filters_per_launch", 0):
        r["profile_check"] = _profile_check("c4", ["k_build_part", "k_build_tile_sub"], per_gpu, r["frac_one_lane"])
    return r


_LANES = None  # the default line's lane streams, made once at its start
WARM_S = 0.3   # a secondary leg's time-based warm-up (warm_up)


def warm_up(torch, dev, step, steps, seconds=WARM_S):
    """A secondary leg's untimed warm-up: at least `steps` steps, and steps
    until `seconds` of wall time have passed, so the chip's clocks have ramped
    whether the leg runs inside the default line (after seconds of other
    legs) or alone in a fresh process (tools/profile_round.sh). C4 alone after
    5 steps ran at 121.5-123.4 us per step against 112.5-113.3 after 3000
    (experiment r05_warm, HISTORY.md); the profiles' one-lane durations were taken that
    way, which round 4 and early round 5 read as box-to-box variation."""
    t0 = time.perf_counter()
    i = 0
    while i < steps or time.perf_counter() - t0 < seconds:
        step()
        i += 1
        if i % 64 == 0:
            torch.cuda.synchronize(dev)  # bounded queue depth, and the elapsed time is the device's
    torch.cuda.synchronize(dev)


def leg_lanes(torch, dev, P):
    """A leg's P pipeline lanes: the line's own lane streams when it has made
    them (every leg of one line on the same streams), else the current stream
    and P - 1 from torch's pool. HIP multiplexes streams onto a few hardware
    queues (GPU_MAX_HW_QUEUES, 4 here) in creation order, and lanes sharing a
    queue run one after the other: the C5 leg on the current stream plus two
    more pool streams drawn after the C4 leg's took 206-208 us per step on
    three lanes, against 188-189 on the line's lanes, on fresh pool streams
    or on hipStreamCreate streams (experiment r05_c5ctx3, HISTORY.md)."""
    if _LANES and len(_LANES) >= P:
        return list(_LANES[:P])
    return [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(P - 1)]


def c5_leg(args, torch, dev, local, world, rank, steps, warmup, lanes_n, check, red_dev, dist, use_dist):
    """BASELINE C5, one rank's slice of the read fan-out (src/lib.rs:129-134
    over 256 tables, 32 per GPU at 8 GPUs): 10M lookups (SURVEY.md §8d C5
    batch over all 256 tables) probed against this rank's 32 filters of
    m = 2^26 (filters 32r .. 32r+31, key(1000 + f, i < 2^19)) through the
    FilterSet, one [32][156250] hit map per step, lanes_n lanes. The
    all-gather that completes C5 at 8 GPUs runs in `--workload c5 --gpus 8`;
    here the step is the per-GPU probe. check: the rank's whole slice against
    the golden SHA-256, and filter 32r's row against the C oracle."""
    import lsmt_amd
    from lsmt_amd import workload
    g = _golden()["c5"] if check else None
    F, m, kpf, n, nf = 32, 1 << 26, 1 << 19, 10_000_000, 256
    r = rank % 8
    filters = []
    for f in range(32 * r, 32 * r + F):
        b = lsmt_amd.BloomFilter(m, device=local)
        b.insert_batch(lsmt_amd.DeviceKeys(torch.from_numpy(workload.c5_filter_keys(f, kpf)).to(dev)))
        filters.append(b)
    look_np = workload.c5_lookups(n, nf, kpf)
    look = torch.from_numpy(look_np).to(dev)
    keys = lsmt_amd.DeviceKeys(look)
    fset = lsmt_amd.FilterSet(m, width=32, device=local)
    fset.assign_all(filters)
    words = (n + 63) // 64
    P = lanes_n
    lanes = leg_lanes(torch, dev, P)
    hits = [torch.zeros((F, words), dtype=torch.int64, device=dev) for _ in range(P)]
    nstep = [0]

    def step():
        i = nstep[0] % P
        nstep[0] += 1
        fset.probe(keys, out=hits[i], stream=lanes[i].cuda_stream)

    warm_up(torch, dev, step, warmup)
    el, ev_ms = _timed_lanes(torch, dist, dev, use_dist, red_dev, lanes, step, steps)
    nstep[0] = 0
    Psaved, P = P, 1
    _, ev1_ms = _timed_lanes(torch, dist, dev, use_dist, red_dev, lanes[:1], step, steps)
    from lsmt_amd import _lib
    path = int(_lib.load().cb_last_path())  # 6: the dense (region-partitioned) probe, 3: k_set_probe
    kern = ["k_dense_part", "k_dense_seg_t", "k_dense_probe"] if path == 6 else ["k_set_probe"]
    kus = _kernel_us(_lib.load(), torch, dev, kern, step, min(steps, 20))  # one lane (P = 1 still)
    P = Psaved
    sectors, rand_reads = _set_sectors(filters, look_np, m, F)
    alg = 64 * sectors + 16 * n + F * n / 8
    us = ev_ms * 1e3 / steps
    ach = alg / (us * 1e-6) / 1e9
    out = {"slice": f"rank {r} of 8: filters {32 * r}..{32 * r + F - 1} of {nf}", "n_keys": n,
           "filters": F, "m_bits": m, "steps": steps, "pipeline_lanes": lanes_n,
           "ms_per_step": round(el / steps * 1e3, 4), "region_us_per_step": round(us, 2),
           "one_lane_us_per_step": round(ev1_ms * 1e3 / steps, 2),
           "value": round(n * F * world / (el / steps), 1), "unit": "probes/s (all GPUs)",
           "path": "dense (k_dense_part + k_dense_seg_t + k_dense_probe: keys partitioned by set region, regions "
                   "staged in LDS)"
                   if path == 6 else "k_set_probe (one random set line per read)",
           "kernels_us": {k: v["avg_us"] for k, v in kus.items()},
           "kernels_us_source": "library HIP events around each launch, one lane",
           "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 4),
                        "frac_one_lane": round(alg / (ev1_ms * 1e-3 / steps) / 1e9 / HBM_PEAK_GBS, 4),
                        "kernel": "+".join(kern), "kernel_avg_us": round(us, 2),
                        "algorithmic_bytes": int(alg),
                        "algorithmic_def": f"64 B x {sectors} distinct sectors + 16n + F*n/8 "
                                           "(SURVEY.md §8d alternative layout)"}}
    traffic = [_pmc_traffic(k, "c5") for k in kern]
    out["roofline"]["traffic"] = sum(traffic) if all(traffic) else None
    out["roofline"]["traffic_source"] = _pmc_source("c5")
    rr = _random_read_roofline()
    if rr and path != 6:
        out["roofline"]["random_read_frac"] = round(rand_reads / (us * 1e-6) / rr, 4)
    out["roofline"]["profile_check"] = _profile_check("c5", kern, alg, out["roofline"]["frac_one_lane"])
    if out["roofline"]["traffic"]:
        out["roofline"]["traffic_over_algorithmic"] = round(out["roofline"]["traffic"] / alg, 3)
    if check:
        torch.cuda.synchronize(dev)
        got = hits[0].cpu().numpy().view(np.uint64)
        good = _sha(got.astype("<u8")) == g["rank_slice_hits_sha256"][r]
        out["golden_slice_bit_exact"] = _all_ranks_true(torch, dist, use_dist, red_dev, good)
        from oracle import oracle
        o = oracle.OracleFilter(m)
        o.insert_fixed(workload.c5_filter_keys(32 * r, kpf))
        row = oracle.probe_fixed([o], look_np, threads=8)
        out["oracle_row_bit_exact"] = _all_ranks_true(torch, dist, use_dist, red_dev,
                                                      bool(np.array_equal(got[0], row[0])))
        out["oracle_sample"] = f"row of filter {32 * r} (all {n} lookups) vs the C oracle"
        del o
        if rank == 0 and world == 1 and not args.no_cpu:
            # the C oracle (byte-per-bit src/bloom.rs, short-circuit) on one
            # thread over a bounded sample of the same batch: the first 2^20
            # lookups against all 32 filters
            refs = []
            for f in range(32 * r, 32 * r + F):
                o = oracle.OracleFilter(m)
                o.insert_fixed(workload.c5_filter_keys(f, kpf))
                refs.append(o)
            smp = 1 << 20
            t0 = time.perf_counter()
            oracle.probe_fixed(refs, look_np[:smp], threads=1)
            tc = time.perf_counter() - t0
            del refs
            out["cpu_baseline"] = {"value": round(smp * F / tc, 1), "unit": "probes/s", "cores": 1, "kind": "port",
                                   "sample": f"first {smp} of the {n} C5 lookups x {F} filters on 1 thread, "
                                             f"{tc:.2f}s"}
    del filters, fset, hits, look, keys
    torch.cuda.synchronize(dev)
    return out


def run_c4(args, torch, dist, world, rank, local, dev, use_dist, result, red_dev):
    """`--workload c4`: the C4 leg alone (strong scaling: 64 filters split over
    the GPUs), one JSON line from rank 0."""
    leg = c4_leg(args, torch, dist, world, rank, local, dev, use_dist, red_dev, args.steps, args.warmup,
                 args.probe_streams, check=args.check, oracle_sample=4 if args.check else 0)
    if rank == 0:
        nf_total, kpf, m = 64, 1 << 18, 1 << 25
        alg = nf_total * (16 * kpf + m / 8)
        el_step = leg["ms_per_step"] * 1e-3
        line = {"metric": "build keys/s (C4: 64 concurrent flush builds x 256K keys, m=2^25)",
                "value": leg["value"], "unit": "keys/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": leg["ms_per_step"],
                "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u32",
                "data": "synthetic (splitmix64 hex keys, SURVEY.md §8d)",
                "config": {"workload": "C4: 64 filters x 2^18 keys -> m=2^25 each, one subset per GPU",
                           "parallelism": "filter-sharded, no collective", "pipeline_lanes": args.probe_streams},
                "algorithmic_bytes_total": int(alg),
                "step_effective_GBps_all_gpus": round(alg / el_step / 1e9, 1),
                "roofline": c4_roofline(leg, world), "c4": leg,
                "cpu_baseline": c4_cpu_baseline(nf_total, kpf, m) if world == 1 and not args.no_cpu else None}
        if args.rehearse_one_gpu:
            line["rehearsal"] = f"{world} ranks on ONE GPU (gloo): checks the N-rank flow, not a scaling measurement"
            line["valid"] = False
        print(json.dumps(line), file=result, flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


def run_leg(args, torch, dist, world, rank, local, dev, use_dist, result, red_dev):
    """`--leg c2|c5|wide`: one secondary leg alone, its dict as the line's
    "build" / "c5" / "wide_fanout" field (the profiling passes' workload; the
    default line runs the same functions)."""
    import lsmt_amd
    from lsmt_amd import _lib, workload
    L = _lib.load()
    lanes = [torch.cuda.current_stream(dev)]
    if args.leg == "c2":  # --build-streams lanes (1: the one-lane profile pass)
        lanes = leg_lanes(torch, dev, args.build_streams)
        out = c2_leg(args, torch, dist, dev, local, world, use_dist, red_dev, max(args.steps, args.leg_steps),
                     args.warmup, lanes, cold=not args.no_cold)
        key = "build"
    elif args.leg == "c5":
        out = c5_leg(args, torch, dev, local, world, rank, args.steps, args.warmup, args.probe_streams,
                     True, red_dev, dist, use_dist)  # golden + oracle row always; the CPU baseline unless --no-cpu
        key = "c5"
    else:
        def timed(fn, k, lanes=lanes):
            return _timed_lanes(torch, dist, dev, use_dist, red_dev, lanes, fn, k)[0]

        def kernel_ms(names, fn, k):
            return _kernel_us(L, torch, dev, names, fn, k)
        out = wide_fanout_leg(args, torch, dev, local, leg_lanes(torch, dev, args.probe_streams), args.steps * 20,
                              timed, kernel_ms, lsmt_amd, workload)
        key = "wide_fanout"
    if rank == 0:
        print(json.dumps({"leg": args.leg, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          key: out}), file=result, flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


def zone_partitioned_leg(args, torch, dev, local, sh, F, m, kpf, n, timed, kernel_ms, probes_per_step,
                         lsmt_amd, workload):
    """Gated FilterSet probe over F range-partitioned tables: the F * kpf
    keys of seed 4000 sorted and cut into F contiguous ranges (table f = the
    f-th range, its ZoneMap = [first, last key]); lookups: half present keys
    (key j of table j mod F), half absent keys. Reports gated probes/s, the
    fraction of Bloom-passing (key, table) pairs the zones reject, and a
    check of the first 64K lookups' gated hits against the oracle's
    zone.contains && may_contain (ob_probe_gated_var)."""
    allk = workload.sort_keys16(workload.key_range(4000, F * kpf))
    parts = [allk[f * kpf:(f + 1) * kpf] for f in range(F)]
    filters = []
    for p in parts:
        b = lsmt_amd.BloomFilter(m, device=local)
        b.insert_batch(lsmt_amd.DeviceKeys(torch.from_numpy(p).to(dev)), stream=sh)
        filters.append(b)
    fset = lsmt_amd.FilterSet(m, width=32 if F <= 32 else 64, device=local)
    fset.assign_all(filters, stream=sh)
    for f, p in enumerate(parts):
        fset.zone_from_keys(f, lsmt_amd.DeviceKeys(torch.from_numpy(p).to(dev)), stream=sh)
    j = np.arange(n // 2 + n % 2)
    look_np = np.empty((n, 16), np.uint8)
    look_np[0::2] = allk[(j % F) * kpf + (j // F) % kpf]
    look_np[1::2] = workload.key_range(4999, n // 2)
    keys = lsmt_amd.DeviceKeys(torch.from_numpy(look_np).to(dev))
    words = (n + 63) // 64
    gated = torch.zeros((F, words), dtype=torch.int64, device=dev)
    plain = torch.zeros((F, words), dtype=torch.int64, device=dev)
    fset.probe(keys, out=plain, stream=sh)

    def step():
        fset.probe(keys, out=gated, stream=sh, gated=True)

    LK = max(args.steps, args.leg_steps)
    for _ in range(args.warmup):
        step()
    el = timed(step, LK)
    prof = kernel_ms(["k_set_probe_gated"], step, LK)
    torch.cuda.synchronize(dev)
    g = gated.cpu().numpy().view(np.uint64)
    pl = plain.cpu().numpy().view(np.uint64)
    bits = lambda a: int(np.unpackbits(a.view(np.uint8)).sum())
    bloom_pass, gate_pass = bits(pl), bits(g)
    out = {"value": round(probes_per_step / (el / LK), 1), "unit": "gated probes/s",
           "ms_per_step": round(el / LK * 1e3, 4), "steps": LK,
           "kernels_us": {k: round(v["avg_us"], 2) for k, v in prof.items()},
           "bloom_pass_pairs": bloom_pass, "gate_pass_pairs": gate_pass,
           "zone_rejected_fraction_of_bloom_pass": round(1 - gate_pass / max(bloom_pass, 1), 4),
           "tables": f"{F} range-partitioned tables of {kpf} keys (sorted key(4000, i) cut in {F})"}
    if not args.no_cpu:  # oracle check on a sample (CPU restatement as the checker only)
        from oracle import oracle
        sample = 1 << 16
        refs = []
        for p in parts:
            o = oracle.OracleFilter(m)
            o.insert_fixed(p)
            refs.append(o)
        zones = [oracle.OracleZone(bytes(p[0]), bytes(p[-1])) for p in parts]
        d = np.ascontiguousarray(look_np[:sample].reshape(-1))
        offs = np.arange(0, 16 * (sample + 1), 16, dtype=np.uint64)
        exp = oracle.probe_gated(refs, zones, d, offs)
        out["oracle_sample_bit_exact"] = bool(np.array_equal(g[:, :sample // 64], exp))
        del refs
    return out


def wide_fanout_leg(args, torch, dev, local, lanes, LK, timed, kernel_ms, lsmt_amd, workload):
    """Database::get at the reference's own shape: 300
    tables as 300 auto-flushes of 1024 entries leave them (keys from a
    shared pool, so later flushes rewrite keys; each table's filter m = 1024
    and its zone map), held in one wide FilterSet (slot = the table's
    position in Vec<SsTable>), and 2^18 lookups (3/4 present) walked newest
    first in ONE launch (cb_set_get_many_fixed over a 320-slot set). At
    m = 1024 with 1024 keys a filter is 86 % ones, so ~75 % of the tables pass
    the Bloom gate for any key and a lookup searches ~100-225 tables: the
    reference's own cost model. Batches alternate over the line's P lanes
    (as the probe and read legs: each lane its own outputs and workspace), so
    one batch's value scan and base64 decode overlap the next batch's walk;
    the one-lane figure is reported beside it. Oracle: the first 4096 lookups
    through the CPU restatement of the same gate and walk, and every lane's
    answers equal."""
    sh = lanes[0].cuda_stream
    P = len(lanes)
    nt, per, n = 300, 1024, 1 << 18
    rng = np.random.default_rng(300)
    pool = workload.key_range(4242, 120_000)
    tables, blooms, zones, ents = [], [], [], []
    t0 = time.perf_counter()
    for t in range(nt):
        idx = np.unique(rng.choice(len(pool), per, replace=False))
        ks = np.ascontiguousarray(pool[idx])
        vs = workload.table_value(ks, t)
        kb = lsmt_amd.KeyBatch(n=len(idx), data=ks.reshape(-1), offsets=np.arange(0, 16 * (len(idx) + 1), 16,
                                                                                 dtype=np.uint64))
        vb = lsmt_amd.KeyBatch(n=len(idx), data=np.ascontiguousarray(vs).reshape(-1),
                               offsets=np.arange(0, 16 * (len(idx) + 1), 16, dtype=np.uint64))
        tb, bloom, zone = lsmt_amd.sstable_create((kb, vb), m=1024, device=local)
        tables.append(tb)
        blooms.append(bloom)
        zones.append(zone)
        ents.append((ks, vs))
    flush_s = time.perf_counter() - t0
    fset = lsmt_amd.FilterSet(1024, width=320, device=local)
    for t in range(nt):
        fset.assign(t, blooms[t])
        fset.set_zone(t, zones[t])
    present = pool[rng.integers(0, len(pool), 3 * n // 4)]
    look_np = np.concatenate([present, workload.key_range(4343, n - len(present))])[rng.permutation(n)]
    keys = lsmt_amd.DeviceKeys(torch.from_numpy(look_np).to(dev))
    newest_first = tables[::-1]
    slots = np.arange(nt, dtype=np.uint32)[::-1].copy()
    which_l = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(P)]
    voff_l = [torch.empty(n + 1, dtype=torch.int64, device=dev) for _ in range(P)]
    vals_l = [torch.empty(n * 16, dtype=torch.uint8, device=dev) for _ in range(P)]
    nxt = [0]

    def lane_step(b):
        lsmt_amd.get_many(newest_first, keys, filterset=fset, hit_rows=slots, out=(which_l[b], voff_l[b], vals_l[b]),
                          stream=lanes[b].cuda_stream, wait=False)

    def step():  # batches round-robin over the lanes
        b = nxt[0] % P
        nxt[0] += 1
        lane_step(b)

    def step1():
        lane_step(0)

    for b in range(P):  # each lane's workspace builds its screen once
        warm_up(torch, dev, lambda: lane_step(b), 2)
    # 100 steps at the default K (12 ms): the host issues a step in ~30 us
    # against ~110 us of device time (tools/wide_issue.py), so the queue runs
    # ahead after the first step; 10 steps left that first step's issue and
    # the box's host jitter in the figure
    k = max(20, LK // 2)
    el1 = timed(step1, k, lanes=lanes[:1])
    el = timed(step, k, lanes=lanes) if P > 1 else el1
    kus = kernel_ms(["k_wide_get_many", "k_tile_scan", "k_b64_decode"], step1, k)
    torch.cuda.synchronize(dev)
    found = int((which_l[0] >= 0).sum().item())
    tot = int(voff_l[0][n].item())  # value bytes written (the buffers' tails are never written)
    lanes_equal = all(torch.equal(which_l[0], w) and torch.equal(voff_l[0], v) and
                      torch.equal(vals_l[0][:tot], x[:tot]) for w, v, x in zip(which_l, voff_l, vals_l))
    which, voff, vals = which_l[0], voff_l[0], vals_l[0]
    out = {"metric": f"gets/s: Database::get over {nt} tables of m=1024 (1024 entries each) in one wide set",
           "value": round(n / (el / k), 1), "unit": "keys/s", "ms_per_step": round(el / k * 1e3, 4), "steps": k,
           "pipeline_lanes": P, "lanes_equal": bool(lanes_equal),
           "one_lane": {"value": round(n / (el1 / k), 1), "ms_per_step": round(el1 / k * 1e3, 4)},
           "tables": nt, "set_width": 320, "lookups": n, "found": found,
           "kernels_us": {kk: round(v["avg_us"], 2) for kk, v in kus.items()},
           "launches_per_batch": {kk.replace("k_", "", 1): round(v["launches"] / k, 2) for kk, v in kus.items()},
           "table_build_s": round(flush_s, 2)}
    # roofline of the search launch: its compulsory HBM bytes are the keys
    # (16 B) and its three per-lookup outputs (which 4 B, value source 8 B,
    # decoded length 8 B), plus one 128-B key-bucket line per found key; the
    # set's rows (40 KB), the screen (1.3 MB) and the summary words (2.4 MB)
    # stay in every XCD's L2. It is bound by dependent L2 round trips (rows ->
    # screen -> summary words of the survivors -> bucket line), not by bytes.
    wk = kus.get("k_wide_get_many", {}).get("avg_us")
    if wk:
        alg = n * (16 + 4 + 8 + 8) + found * 128
        wr = {"bound": "latency (dependent L2 round trips per lookup)", "kernel": "k_wide_get_many",
              "kernel_avg_us": wk, "algorithmic_bytes": int(alg),
              "algorithmic_def": "n x (16 B key + 20 B outputs) + 128 B bucket line per found key",
              "achieved": round(alg / (wk * 1e-6) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "frac": round(alg / (wk * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
        name, d = _pmc_summary("wide")
        e = (d or {}).get("kernels", {}).get("k_wide_get_many", {})
        if e.get("hbm_bytes_per_launch"):
            wr["traffic"] = int(e["hbm_bytes_per_launch"])
            wr["traffic_source"] = f"profiles/{name}"
            if e.get("TCC_HIT_sum") is not None and e.get("TCC_MISS_sum") is not None:
                req = e["TCC_HIT_sum"] + e["TCC_MISS_sum"]
                wr["l2_requests_per_launch"] = int(req)
                wr["l2_hit_rate"] = round(e["TCC_HIT_sum"] / req, 4) if req else None
                wr["l2_requests_per_lookup"] = round(req / n, 1)
            if e.get("avg_us_one_lane"):
                wr["profile_check"] = {"source": f"profiles/{name} (rocprofv3 --kernel-trace)",
                                       "kernel_us": e["avg_us_one_lane"],
                                       "ratio_to_line_kernel_us": round(wk / e["avg_us_one_lane"], 4)}
        out["roofline"] = wr
    if not args.no_cpu:
        from oracle import oracle
        smp = 4096
        d = np.ascontiguousarray(look_np[:smp].reshape(-1))
        offs = np.arange(0, 16 * (smp + 1), 16, dtype=np.uint64)
        ofs, ozs, ots = [], [], []
        for t in range(nt - 1, -1, -1):
            o = oracle.OracleFilter(1024)
            o.insert_fixed(ents[t][0])
            ofs.append(o)
            ozs.append(oracle.OracleZone(zones[t].min, zones[t].max))
            ots.append(oracle.OracleTable(tables[t].data()))
        t0 = time.perf_counter()
        gate = oracle.probe_gated(ofs, ozs, d, offs)
        ow, ovoff, ovals = oracle.get_many(ots, gate, d, offs)
        tc = time.perf_counter() - t0
        gvo = voff[: smp + 1].cpu().numpy().astype(np.uint64)
        out["oracle_sample_bit_exact"] = bool(
            np.array_equal(which[:smp].cpu().numpy(), ow) and np.array_equal(gvo, ovoff) and
            bytes(vals[: int(gvo[-1])].cpu().numpy()) == ovals)
        out["cpu_baseline"] = {"value": round(smp / tc, 1), "unit": "keys/s", "cores": 1, "kind": "port",
                               "sample": f"oracle gate + newest-first walk over {nt} tables for the first {smp} "
                                         f"lookups, {tc:.2f}s"}
    del tables, blooms, fset, keys, which, voff, vals, which_l, voff_l, vals_l
    torch.cuda.synchronize(dev)
    return out


def may_contain_latency():
    """tests/cpp/may_contain_latency (plain C over include/cassbloom.h, built
    by __graft_entry__.build()): per-key cb_may_contain from one host thread,
    the host mirror (steady state and the first call after the build) against
    a one-key GPU probe per call; the two agree on every probe key."""
    exe = os.path.join(ROOT, "build", "tests", "may_contain_latency")
    if not os.path.exists(exe):  # (a tree without the prebuilt tools: gcc over the header and the .so)
        try:
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True,
                           capture_output=True, timeout=120)
        except Exception as e:  # reported in the line, never fatal to the headline
            return {"error": f"building tests/cpp/may_contain_latency failed: {e!r}"[:300]}
    out = {"metric": "single-key may_contain latency, one host thread, C ABI (SsTable::get's per-table "
                     "bloom.may_contain, src/sstable.rs:138)"}
    for label, m, nk in (("m1024", 1024, 100), ("m2^26", 1 << 26, 1 << 19)):
        try:
            r = subprocess.run([exe, str(m), str(nk), "400000"], capture_output=True, text=True, timeout=120)
            d = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {"error": r.stderr[-400:]}
        except Exception as e:  # reported in the line, never fatal to the headline
            d = {"error": repr(e)}
        out[label] = d
    return out


def _set_sectors(filters, look_np, m, F):
    """Compulsory reads of one FilterSet probe batch (k_set_probe): set[a] for
    every key and set[b] where set[a] != 0 (with CB_SET_ANY=1: any[a], any[b]
    for every key and set[a], set[b] for keys passing the union test).
    Returns (distinct 64-B sectors touched, number of random set-word reads),
    from the filters' packed words and a numpy restatement of the hashes."""
    anyw = np.zeros((m + 31) // 32, np.uint32)
    for f in filters:
        anyw |= f.packed()
    h1 = np.full(look_np.shape[0], 5381, np.uint64)
    h2 = np.zeros(look_np.shape[0], np.uint64)
    with np.errstate(over="ignore"):
        for j in range(look_np.shape[1]):
            b = look_np[:, j].astype(np.uint64)
            h1 = (h1 << np.uint64(5)) + h1 + b
            h2 = h2 * np.uint64(31) + b
    a = (h1 % np.uint64(m)).astype(np.int64)
    bpos = (h2 % np.uint64(m)).astype(np.int64)
    bit = lambda p: ((anyw[p >> 5] >> (p & 31).astype(np.uint32)) & 1).astype(bool)
    word_bytes = 4 if F <= 32 else 8
    if os.environ.get("CB_SET_ANY") == "1":  # union pre-test mode
        passed = bit(a) & bit(bpos)
        set_sec = np.concatenate([(a[passed] * word_bytes) >> 6, (bpos[passed] * word_bytes) >> 6])
        any_sec = np.concatenate([a >> 9, bpos >> 9])  # 512 positions per 64-B sector of any[]
        return int(np.unique(set_sec).size) + int(np.unique(any_sec).size), int(set_sec.size)
    # default: set[a] for every key, set[b] only where set[a] != 0 (short-circuit)
    set_sec = np.concatenate([(a * word_bytes) >> 6, (bpos[bit(a)] * word_bytes) >> 6])
    return int(np.unique(set_sec).size), int(set_sec.size)


def _random_read_roofline():
    """Measured MI355X random 4-byte read rate on a 256 MiB table (the set's
    size), from tools/ubench_random.hip's committed output."""
    try:
        with open(os.path.join(ROOT, "profiles", "ubench_random_r01.json")) as fh:
            d = json.load(fh)
        for r in d["random_reads"]:
            if r["table_MiB"] == 256 and r["mem"] == "hipMalloc":
                return float(r["reads_per_s"])
    except Exception:
        return None
    return None


PMC_INDEX = os.path.join(ROOT, "profiles", "pmc_index.json")


def _pmc_summary(shape):
    """(file name, summary dict) of the PMC summary profiles/pmc_index.json
    names for `shape` ("c3", "c4", "c5", "wide"): an explicit choice per
    round, not the newest-looking file name (a lexicographic sort
    picked pmc_r04a over pmc_r04). (None, None) when the shape has none."""
    try:
        with open(PMC_INDEX) as fh:
            name = json.load(fh).get(shape)
        if not name:
            return None, None
        with open(os.path.join(ROOT, "profiles", name)) as fh:
            return name, json.load(fh)
    except Exception:
        return None, None


def _pmc_field(shape, key, default):
    """A top-level field of the shape's indexed PMC summary."""
    _, d = _pmc_summary(shape)
    return d.get(key, default) if d else default


def _pmc_traffic(kernel, shape="c3"):
    """HBM bytes per launch of `kernel` from the shape's indexed rocprofv3 PMC
    summary (FETCH_SIZE/WRITE_SIZE priced per request size, the gfx950
    corrections of tools/pmc_summary.py), or None when none was recorded."""
    _, d = _pmc_summary(shape)
    if not d:
        return None
    v = d.get("kernels", {}).get(kernel, {}).get("hbm_bytes_per_launch")
    return int(v) if v else None


def _pmc_source(shape):
    name, _ = _pmc_summary(shape)
    return f"profiles/{name}" if name else None


def _profile_check(shape, kernels, alg_bytes, line_frac_one_lane):
    """The roofline fraction recomputed from the shape's committed rocprofv3
    one-lane trace (the sum of `kernels`' average one-lane dispatch durations
    = one step) beside the line's own one-lane (HIP-event) fraction: the two
    clocks, and their ratio (within 3 %)."""
    name, d = _pmc_summary(shape)
    if not d:
        return None
    ks = d.get("kernels", {})
    us = [ks.get(k, {}).get("avg_us_one_lane") for k in kernels]
    if not all(us):
        return None
    step = sum(us)
    frac = alg_bytes / (step * 1e-6) / 1e9 / HBM_PEAK_GBS
    out = {"source": f"profiles/{name} (rocprofv3 --kernel-trace, one lane)", "kernels": list(kernels),
           "step_us": round(step, 2), "frac": round(frac, 4)}
    ev = d.get("events_one_lane_us", {})
    if ev.get("traced"):  # the same traced run's own HIP-event step: the two clocks on one run
        out["traced_run_events_us"] = ev["traced"]
        out["ratio_to_traced_run_events"] = round(ev["traced"] / step, 4)
    if ev.get("plain"):  # the profiled box's untraced run of the same command
        out["plain_run_events_us"] = ev["plain"]
    if line_frac_one_lane:
        out["ratio_to_line_frac_one_lane"] = round(frac / line_frac_one_lane, 4)
    return out


def c4_cpu_baseline(nf, kpf, m):
    """SURVEY.md §8d CPU baseline for C4: the C oracle (byte-per-bit
    src/bloom.rs) building the 64 filters one after another on one thread,
    and over 16 threads (one filter per task; ctypes releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor

    from lsmt_amd import workload
    from oracle import oracle
    keys = [workload.c4_filter_keys(f, kpf) for f in range(nf)]

    def build(k):
        o = oracle.OracleFilter(m)
        o.insert_fixed(k)
        del o

    t0 = time.perf_counter()
    for k in keys:
        build(k)
    t1 = time.perf_counter() - t0
    cpus = host_cpus()
    threads = cpus["usable"]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(build, keys))
    tn = time.perf_counter() - t0
    return {"value": round(nf * kpf / t1, 1), "unit": "keys/s", "cores": 1, "kind": "port",
            "sample": f"all {nf} C4 builds ({kpf} keys -> m=2^{m.bit_length() - 1} bytes each) on 1 thread, {t1:.2f}s",
            "all_cores": {"value": round(nf * kpf / tn, 1), "threads": threads, "seconds": round(tn, 3),
                          "note": cpus["note"]}}


def cpu_baseline(look_np, F, m, kpf, build_keys, build_m):
    """The C oracle (byte-per-bit restatement of src/bloom.rs, short-circuit
    probe) on this host's cores: the full C3 probe (1M keys x F filters) on one
    thread, the same on all cores, and the C2 build on one thread."""
    from lsmt_amd import workload
    from oracle import oracle
    refs = []
    for f in range(F):
        o = oracle.OracleFilter(m)
        o.insert_fixed(workload.key_range(100 + f, kpf))
        refs.append(o)
    n = look_np.shape[0]
    reps = 3  # ~10 s of single-thread CPU work in all
    t0 = time.perf_counter()
    for _ in range(reps):
        oracle.probe_fixed(refs, look_np, threads=1)
    t1 = (time.perf_counter() - t0) / reps
    cpus = host_cpus()
    cores = cpus["usable"]
    t0 = time.perf_counter()
    oracle.probe_fixed(refs, look_np, threads=cores)
    tn = time.perf_counter() - t0
    del refs
    # C2 build on one thread: repeated until at least 1 s of build time
    # (one rep is ~25 ms), each rep into a fresh zeroed filter
    bk = workload.c2_build_keys(build_keys)
    tb_sum, breps = 0.0, 0
    while tb_sum < 1.0 or breps < 3:
        o = oracle.OracleFilter(build_m)
        t0 = time.perf_counter()
        o.insert_fixed(bk)
        tb_sum += time.perf_counter() - t0
        breps += 1
        del o
    tb = tb_sum / breps
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(n * F / t1, 1), "unit": "probes/s", "cores": 1, "kind": "port",
            "sample": f"full C3 probe: {n} keys x {F} filters (m=2^{m.bit_length() - 1}, byte-per-bit) on 1 thread, "
                      f"{reps} reps of {t1:.2f}s",
            "all_cores": {"value": round(n * F / tn, 1), "threads": cores, "seconds": round(tn, 3),
                          "note": cpus["note"]},
            "build": {"value": round(build_keys / tb, 1), "unit": "keys/s", "cores": 1,
                      "sample": f"C2 build {build_keys} keys into m=2^{build_m.bit_length() - 1} bytes, "
                                f"{breps} reps of {tb:.3f}s ({tb_sum:.2f}s in all)"},
            "cpu_model": cpu_model, "nproc": os.cpu_count(), "cpus": cpus}


def host_cpus():
    """CPUs this process can actually run on: os.cpu_count() (the machine),
    the affinity mask, and the cgroup CPU quota (cpu.max). The all-cores
    baseline uses min(affinity, quota) threads: on a shared GPU box nproc
    counts the whole host while the job is limited to its share."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as fh:
                q, p = fh.read().split()[:2]
                if q != "max":
                    quota = max(1, int(int(q) / int(p)))
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
                q = int(fh.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
                p = int(fh.read())
            if q > 0:
                quota = max(1, q // p)
        except (OSError, ValueError):
            pass
    usable = min(aff, quota) if quota else aff
    # the GPU box declares the job's CPU share in OMP_NUM_THREADS (16 per GPU)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    share = int(omp) if omp.isdigit() and int(omp) > 0 else None
    if share:
        usable = min(usable, share)
    note = (f"threads = CPUs this job may use: nproc {nproc} (whole host), affinity {aff}, cgroup quota "
            f"{quota if quota else 'none'}, OMP_NUM_THREADS {share if share else 'unset'}")
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "omp_share": share, "usable": usable,
            "note": note}


if __name__ == "__main__":
    main()
