"""One process per GPU: rendezvous, sharding and whole-job timing for batch sealing.

Records are independent, so a multi-GPU job is N copies of the single-GPU path over disjoint
shards of the record stream (workload.shard_batch): no collective touches the data. The only
collectives are the barriers around the timed region and one max-reduce of the wall time
(torch.distributed; backend "nccl" = RCCL on ROCm between GPUs, "gloo" for CPU tests).
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
    kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
    tdist.init_process_group(backend, **kw)
    return True


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


def scatter_gather(nbytes, device=None, reps=3):
    """Time the exchange the bulk path needs when a batch arrives at one rank:
    rank 0 scatters `nbytes` of records to every rank and gathers `nbytes` of sealed output back
    (torch.distributed scatter / gather: RCCL over xGMI for "nccl", gloo on CPU). Not on the
    timed sealing path. Returns (scatter_GBps, gather_GBps) of the bytes leaving / entering rank
    0 for the other ranks, max time over ranks, or None for a single rank."""
    if not (tdist.is_available() and tdist.is_initialized()):
        return None
    rank, world = tdist.get_rank(), tdist.get_world_size()
    buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
    parts = [torch.full((nbytes,), r, dtype=torch.uint8, device=device) for r in range(world)] if rank == 0 else None

    def sync():
        if device is not None and device.type == "cuda":
            torch.cuda.synchronize(device)

    def timed(fn):
        fn()  # warm-up (communicator, buffers)
        sync()
        barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        sync()
        return max_over_ranks((time.perf_counter() - t0) / reps, device)

    ts = timed(lambda: tdist.scatter(buf, scatter_list=parts, src=0))
    if not bool((buf == rank).all()):
        raise RuntimeError("scatter delivered the wrong shard")
    tg = timed(lambda: tdist.gather(buf, gather_list=parts, dst=0))
    moved = (world - 1) * nbytes / 1e9
    return moved / ts, moved / tg


def close():
    if tdist.is_available() and tdist.is_initialized():
        barrier()
        tdist.destroy_process_group()
