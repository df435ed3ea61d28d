"""Multi-rank path on CPU (world size 2, gloo): shards are disjoint slices of the config's record
stream, the per-rank results of the sealing step (here the oracle, standing in for the GPU) put
together equal the unsharded batch's, and the timing helpers (barriers + max over ranks)
behave as bench.py relies on."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_PER_RANK = 24
CONFIG = "c5_mixed_256Ki_x_64B-16KiB"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _seal_shard(batch, seed):
    import oracle as ora
    from test_gpu_parity import oracle_keys, oracle_recs

    rng = np.random.default_rng(seed)
    inbuf = rng.integers(0, 256, size=batch["in_bytes"] + 16, dtype=np.uint8)
    out = np.zeros(batch["out_bytes"] + 16, np.uint8)
    tags = np.zeros(16 * len(batch["recs"]), np.uint8)
    assert ora.seal_batch(oracle_keys(batch["keys"]), oracle_recs(batch["recs"]), inbuf, np.zeros(16, np.uint8),
                          out, tags, 1) == 0
    return inbuf, out, tags


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), ATLS_NO_TORCH_RUNTIME="1")
    import torch.distributed as tdist

    from anothertls_amd import dist, workload

    assert dist.init("gloo")
    batch = workload.shard_batch(CONFIG, rank, n=N_PER_RANK)
    inbuf, out, tags = _seal_shard(batch, 100 + rank)
    calls = []
    wall = dist.timed_steps(lambda: calls.append(1), steps=5, warmup=2, sync=lambda: None)
    # rank 1 reports a longer time: the max must win on every rank
    mx = dist.max_over_ranks(1.0 + rank)
    # bench.py's scatter/gather timing (RCCL on the GPU box): shards arrive intact, rates > 0
    sg = dist.scatter_gather(1 << 16)
    assert sg is not None and sg[0] > 0 and sg[1] > 0
    gathered = [None] * world
    tdist.all_gather_object(gathered, (batch["recs"].tobytes(), inbuf.tobytes(), out.tobytes(), tags.tobytes()))
    q.put((rank, len(calls), wall, mx, gathered if rank == 0 else None))
    dist.close()


@pytest.mark.timeout(300)
def test_two_rank_shards_match_unsharded_batch():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    for rank, ncalls, wall, mx, _ in res:
        assert ncalls == 7 and wall >= 0.0 and mx == 2.0, (rank, ncalls, wall, mx)
    gathered = res[0][4]

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from anothertls_amd import REC_DTYPE, workload

    full = workload.config_batch(CONFIG, n=world * N_PER_RANK)
    recs = [np.frombuffer(g[0], REC_DTYPE) for g in gathered]
    for f in ("len", "key_slot", "seq", "content_type", "mode"):
        assert np.array_equal(np.concatenate([r[f] for r in recs]), full["recs"][f]), f
    # the unsharded batch sealed with the shards' payloads gives the shards' tags and bytes
    for rank, g in enumerate(gathered):
        shard = workload.shard_batch(CONFIG, rank, n=N_PER_RANK)
        inbuf = np.frombuffer(g[1], np.uint8)
        _, out, tags = _seal_shard(shard, 100 + rank)
        assert np.frombuffer(g[3], np.uint8).tobytes() == tags.tobytes()
        assert np.frombuffer(g[2], np.uint8).tobytes() == out.tobytes()
        # and each shard record equals the same record sealed inside the full batch
        sub = dict(full)
        lo = rank * N_PER_RANK
        sub_recs = full["recs"][lo:lo + N_PER_RANK].copy()
        sub_recs["in_off"] = shard["recs"]["in_off"]
        sub_recs["out_off"] = shard["recs"]["out_off"]
        sub = dict(keys=full["keys"], recs=sub_recs, in_bytes=shard["in_bytes"], out_bytes=shard["out_bytes"])
        _, out2, tags2 = _seal_shard_with(sub, inbuf)
        assert tags2.tobytes() == tags.tobytes() and out2.tobytes() == out.tobytes()


def _seal_shard_with(batch, inbuf):
    import oracle as ora
    from test_gpu_parity import oracle_keys, oracle_recs

    out = np.zeros(batch["out_bytes"] + 16, np.uint8)
    tags = np.zeros(16 * len(batch["recs"]), np.uint8)
    assert ora.seal_batch(oracle_keys(batch["keys"]), oracle_recs(batch["recs"]), inbuf, np.zeros(16, np.uint8),
                          out, tags, 1) == 0
    return inbuf, out, tags
