"""One process per GPU: rendezvous, sharding and whole-job timing for batch sealing.

Records are independent, so a multi-GPU job is N copies of the single-GPU path over disjoint
shards of the record stream (workload.shard_batch): no collective touches the data of the timed
path. Its only collectives are the barriers around the timed region and one max-reduce of the
wall time (torch.distributed; backend "nccl" = RCCL on ROCm between GPUs, "gloo" for CPU tests).
A batch that arrives at one rank is spread with seal_sharded: a byte-balanced split, RCCL
point-to-point scatter of the record ranges, per-rank sealing and a gather back.
"""
import os
import time

import torch
import torch.distributed as tdist


def env_ranks():
    """(rank, local_rank, world_size) from the torch.distributed.run environment."""
    return int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


def init(backend, device=None):
    """Join the process group (MASTER_ADDR defaults to 127.0.0.1). No-op for a single rank."""
    _, _, world = env_ranks()
    if world <= 1:
        return False
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    import datetime

    kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
    # every collective here takes seconds at most: fail instead of hanging a benchmark run
    tdist.init_process_group(backend, timeout=datetime.timedelta(seconds=300), **kw)
    return True


def world_size():
    """World size of the joined process group (1 when there is none)."""
    return tdist.get_world_size() if (tdist.is_available() and tdist.is_initialized()) else 1


def launch_ranks(argv, n, timeout_s=None):
    """Start n copies of `argv` (a Python script and its arguments) as rank processes on this
    node -- RANK = LOCAL_RANK = 0..n-1, WORLD_SIZE = n, MASTER_ADDR 127.0.0.1 and a free port, as
    torch.distributed.run sets them -- and wait for them. The caller must not have touched the GPU
    (each rank is a fresh process that opens its own device). When a rank fails, the others are
    ended (by their own PIDs). Returns the first non-zero exit status, else 0."""
    import signal
    import socket
    import subprocess
    import sys

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, *argv], env=env))
    status, t0 = 0, time.monotonic()
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
        if status or (timeout_s is not None and time.monotonic() - t0 > timeout_s):
            for p in live:  # a failed or overdue rank: end the others, then collect them
                p.send_signal(signal.SIGTERM)
            for p in live:
                try:
                    p.wait(30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            if not status:
                status = WATCHDOG_EXIT
            break
        time.sleep(0.05)
    return status


def barrier():
    if tdist.is_available() and tdist.is_initialized():
        tdist.barrier()


def max_over_ranks(x, device=None):
    """Max of a float over all ranks (the job ends when its slowest rank does)."""
    if not (tdist.is_available() and tdist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())


def timed_steps(step, steps, warmup, sync, device=None):
    """Run `warmup` untimed steps, then time exactly `steps` steps between barrier + sync on
    both sides; returns the max wall time over ranks (seconds)."""
    for _ in range(warmup):
        step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    t1 = time.perf_counter()
    barrier()
    return max_over_ranks(t1 - t0, device)


def whole_job_rate(bytes_per_rank, steps, wall, world):
    """Aggregate GiB/s: every rank processes bytes_per_rank per step (weak scaling)."""
    return world * bytes_per_rank * steps / wall / 2**30


def extents(recs, open_=False):
    """Per record: bytes read at in_off and written at out_off (include/atls.h modes: TLS seal
    writes content + type byte, WIRE seal header || ct || tag, WIRE open reads the wire record)."""
    import numpy as np

    L = recs["len"].astype(np.int64)
    mode = recs["mode"]
    if open_:
        return np.where(mode == 2, L + 21, L), L
    return L, np.where(mode == 1, L, np.where(mode == 2, L + 22, L + 1))


# Largest point-to-point message: RCCL 2.26 (the librccl PyTorch ships here) returned wrong bytes past the
# first GiB of a single 2 GiB send / recv (tools/multi_diag.py, profiles/r04/multi_diag.log: every record
# in the second half of each 2 GiB C4 range), so ranges travel in pieces of at most 1 GiB, matched in
# order on both sides. csrc/multi.cpp cuts its RCCL transfers the same way.
P2P_PIECE = 1 << 30


def _pieces(t):
    n = t.numel()
    return [t[o:o + P2P_PIECE] for o in range(0, n, P2P_PIECE)] or [t]


def isend_pieces(t, dst):
    return [tdist.isend(p, dst=dst) for p in _pieces(t)]


def irecv_pieces(t, src):
    return [tdist.irecv(p, src=src) for p in _pieces(t)]


def seal_sharded(seal, recs, inp=None, out=None, tags=None, device=None):
    """Seal one batch that arrives at rank 0 with every rank's GPU: the records are cut into
    contiguous ranges balanced by cumulative bytes (atls_partition, the split the C ABI's
    atls_multi_* uses), rank 0 sends each rank its range's input bytes (and its output range, so
    bytes between records survive), every rank seals its range with `seal(recs, inp, out, tags)`
    on rebased descriptors (rank 0 in place), and the sealed ranges and tags come back into
    rank 0's `out` / `tags`. Point-to-point torch.distributed (RCCL over xGMI for "nccl", gloo
    on CPU). `recs` (the numpy descriptors) on every rank; the tensors on rank 0 only. Ranges
    must increase with the record index, as in atls_multi_*. Returns this rank's record range."""
    import numpy as np

    import anothertls_amd as atls

    initialized = tdist.is_available() and tdist.is_initialized()
    rank, world = (tdist.get_rank(), tdist.get_world_size()) if initialized else (0, 1)
    first = atls.partition(recs, world)
    ilen, olen = extents(recs)

    def span(r):
        a, b = int(first[r]), int(first[r + 1])
        if a == b:
            return a, b, 0, 0, 0, 0
        return (a, b, int(recs["in_off"][a]), int(recs["in_off"][b - 1]) + int(ilen[b - 1]),
                int(recs["out_off"][a]), int(recs["out_off"][b - 1]) + int(olen[b - 1]))

    a, b, in_lo, in_hi, out_lo, out_hi = span(rank)
    if rank == 0:
        reqs = []
        for r in range(1, world):
            ra, rb, ilo, ihi, olo, ohi = span(r)
            if ra < rb:
                reqs += isend_pieces(inp[ilo:ihi], r) + isend_pieces(out[olo:ohi], r)
        if a < b:
            seal(recs[a:b], inp, out, tags[16 * a:16 * b])
        for q in reqs:
            q.wait()
        reqs = []
        for r in range(1, world):
            ra, rb, ilo, ihi, olo, ohi = span(r)
            if ra < rb:
                reqs += irecv_pieces(out[olo:ohi], r) + irecv_pieces(tags[16 * ra:16 * rb], r)
        for q in reqs:
            q.wait()
    elif a < b:
        import torch

        loc_in = torch.empty(in_hi - in_lo, dtype=torch.uint8, device=device)
        loc_out = torch.empty(out_hi - out_lo, dtype=torch.uint8, device=device)
        loc_tags = torch.empty(16 * (b - a), dtype=torch.uint8, device=device)
        for q in irecv_pieces(loc_in, 0) + irecv_pieces(loc_out, 0):
            q.wait()
        local = recs[a:b].copy()
        local["in_off"] -= np.uint64(in_lo)
        local["out_off"] -= np.uint64(out_lo)
        seal(local, loc_in, loc_out, loc_tags)
        for q in isend_pieces(loc_out, 0) + isend_pieces(loc_tags, 0):
            q.wait()
    return a, b


WATCHDOG_EXIT = 3  # status of a process whose watchdog fired (a hung step is a failure, not success)


def run_or_exit(fn, timeout_s, on_timeout, status=None):
    """fn() with a watchdog: if it has not returned after timeout_s seconds, on_timeout() runs
    (e.g. print the result gathered so far) and the process exits with status WATCHDOG_EXIT -- for
    steps after a benchmark's timed region whose collectives could hang (the measured line is
    still printed, and the non-zero status says something hung). Returns (True, fn's value) or
    (False, the exception fn raised). status: the exit status instead of WATCHDOG_EXIT."""
    import threading

    lock, state = threading.Lock(), {"done": False}

    def fire():
        with lock:
            if state["done"]:
                return
            state["done"] = True
            try:
                on_timeout()
            finally:
                os._exit(WATCHDOG_EXIT if status is None else status)

    timer = threading.Timer(timeout_s, fire)
    timer.daemon = True
    timer.start()
    try:
        res = (True, fn())
    except Exception as exc:  # noqa: BLE001 -- reported to the caller
        res = (False, exc)
    with lock:
        state["done"] = True
        timer.cancel()
    return res


COMMS_EXIT = 4  # status of a rank whose process group could not run its first collective


def check_comms(device=None, timeout_s=120.0, what="RCCL"):
    """The process group's first collective (a one-element all-reduce and a barrier; with backend "nccl" this is
    where RCCL builds its communicator between the GPUs), under a watchdog: if it raises, or has not finished
    after timeout_s, the rank prints why to stderr and exits with COMMS_EXIT -- a clear refusal instead of a
    benchmark that hangs in its first barrier. No-op without a process group.
    ATLS_TEST_COMMS_FAIL=raise|hang (tests/test_bench_launch.py) makes rank 1 fail that way instead."""
    if not (tdist.is_available() and tdist.is_initialized()):
        return
    import sys

    rank, world = tdist.get_rank(), tdist.get_world_size()

    def refuse(why):
        print(f"bench.py: rank {rank} of {world}: {what} between the ranks failed at its first collective: {why}",
              file=sys.stderr, flush=True)

    def first_collective():
        inject = os.environ.get("ATLS_TEST_COMMS_FAIL")
        if inject and rank == 1:
            if inject == "hang":
                time.sleep(10 * timeout_s)
            raise RuntimeError(f"injected failure ({inject})")
        t = torch.ones(1, dtype=torch.float64, device=device)
        tdist.all_reduce(t)
        if int(t.item()) != world:
            raise RuntimeError(f"all-reduce of ones gave {t.item()}, not {world}")
        tdist.barrier()

    ok, err = run_or_exit(first_collective, timeout_s, lambda: refuse(f"no answer within {timeout_s:.0f} s"),
                          status=COMMS_EXIT)
    if not ok:
        refuse(f"{type(err).__name__}: {str(err)[:300]}")
        os._exit(COMMS_EXIT)


def close():
    if tdist.is_available() and tdist.is_initialized():
        barrier()
        tdist.destroy_process_group()
