"""Multi-rank path on CPU (world size 2, gloo): a batch that arrives at rank 0 is split by
cumulative bytes (atls_partition), scattered, sealed per rank and gathered back by
dist.seal_sharded -- here with the oracle as each rank's sealer, so the exchange logic runs on CPU
(tests/test_gpu_dist.py runs the same function with the real engine on the GPU box) -- and the
result equals the unsharded batch byte for byte, gaps between records included. Also the timing
helpers (barriers + max over ranks) bench.py relies on."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_RECORDS = 48
CONFIG = "c5_mixed_256Ki_x_64B-16KiB"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_sealer(keys):
    import oracle as ora

    okeys = (ora.OraKey * len(keys)).from_buffer_copy(keys.tobytes())

    def seal(recs, inp, out, tags):
        orecs = (ora.OraRec * len(recs)).from_buffer_copy(recs.tobytes())
        assert ora.seal_batch(okeys, orecs, inp.numpy(), np.zeros(16, np.uint8), out.numpy(), tags.numpy(), 1) == 0

    return seal


def _payload(batch):
    return np.random.default_rng(7).integers(0, 256, size=batch["in_bytes"] + 16, dtype=np.uint8)


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), ATLS_NO_TORCH_RUNTIME="1")
    import torch

    from anothertls_amd import dist, workload

    assert dist.init("gloo")
    dist.P2P_PIECE = 777  # every range goes in several point-to-point pieces (the 1 GiB cap, scaled down)
    batch = workload.config_batch(CONFIG, n=N_RECORDS)
    inp = out = tags = None
    if rank == 0:
        inp = torch.from_numpy(_payload(batch))
        out = torch.full((batch["out_bytes"] + 16,), 0xA5, dtype=torch.uint8)  # gap bytes must survive
        tags = torch.zeros(16 * N_RECORDS, dtype=torch.uint8)
    a, b = dist.seal_sharded(_oracle_sealer(batch["keys"]), batch["recs"], inp, out, tags)
    calls = []
    wall = dist.timed_steps(lambda: calls.append(1), steps=5, warmup=2, sync=lambda: None)
    mx = dist.max_over_ranks(1.0 + rank)  # rank 1 reports a longer time: the max must win everywhere
    q.put((rank, a, b, len(calls), wall, mx,
           (out.numpy().tobytes(), tags.numpy().tobytes()) if rank == 0 else None))
    dist.close()


@pytest.mark.timeout(300)
def test_two_rank_sharded_seal_matches_unsharded_batch():
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
    for rank, a, b, ncalls, wall, mx, _ in res:
        assert ncalls == 7 and wall >= 0.0 and mx == 2.0, (rank, ncalls, wall, mx)
    # the two ranges tile the batch and are balanced by bytes, not by count
    assert res[0][1] == 0 and res[0][2] == res[1][1] and res[1][2] == N_RECORDS

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch

    from anothertls_amd import workload

    batch = workload.config_batch(CONFIG, n=N_RECORDS)
    L = batch["recs"]["len"].astype(np.int64)
    cut = res[0][2]
    assert abs(int(L[:cut].sum()) - int(L[cut:].sum())) <= int(L.max()) + 64
    out = torch.full((batch["out_bytes"] + 16,), 0xA5, dtype=torch.uint8)
    tags = torch.zeros(16 * N_RECORDS, dtype=torch.uint8)
    _oracle_sealer(batch["keys"])(batch["recs"], torch.from_numpy(_payload(batch)), out, tags)
    got_out, got_tags = res[0][6]
    assert got_tags == tags.numpy().tobytes()
    assert got_out == out.numpy().tobytes()


def test_partition_balances_cumulative_bytes():
    import anothertls_amd as atls
    from anothertls_amd import workload

    b = workload.config_batch(CONFIG, n=32768)
    L = b["recs"]["len"].astype(np.int64) * 2 + 17
    for parts in (1, 2, 3, 8):
        first = atls.partition(b["recs"], parts)
        assert first[0] == 0 and first[-1] == len(L) and (np.diff(first) >= 0).all()
        share = np.array([L[first[i]:first[i + 1]].sum() for i in range(parts)])
        assert share.max() - share.min() <= 2 * 16401, (parts, share)
    # C4-like equal records: equal counts
    c4 = workload.config_batch("c4_aes256gcm_1Mi_x_16KiB", n=8 * 1000)
    assert (np.diff(atls.partition(c4["recs"], 8)) == 1000).all()
    # more parts than records: empty parts, still a tiling
    f = atls.partition(b["recs"][:3], 8)
    assert f[0] == 0 and f[-1] == 3 and (np.diff(f) >= 0).all()


def test_run_or_exit_watchdog():
    """bench.py's guard around the post-timing exchange (dist.run_or_exit): a step that returns
    or raises is reported; one that hangs ends the process after the timeout with the non-zero
    status dist.WATCHDOG_EXIT, once the timeout callback (bench.py: print the bench line) has run."""
    import subprocess

    code = (
        "import sys, time; sys.path.insert(0, %r)\n"
        "from anothertls_amd import dist\n"
        "print(dist.run_or_exit(lambda: 7, 5, lambda: print('LATE')))\n"
        "ok, exc = dist.run_or_exit(lambda: 1 / 0, 5, lambda: print('LATE'))\n"
        "print(ok, type(exc).__name__)\n"
        "dist.run_or_exit(lambda: time.sleep(60), 0.5, lambda: print('LINE', flush=True))\n"
        "print('NOT REACHED')\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    from anothertls_amd import dist

    assert r.returncode == dist.WATCHDOG_EXIT != 0, (r.returncode, r.stderr)
    assert r.stdout.split("\n")[:3] == ["(True, 7)", "False ZeroDivisionError", "LINE"], r.stdout
    assert "NOT REACHED" not in r.stdout and "LATE" not in r.stdout
