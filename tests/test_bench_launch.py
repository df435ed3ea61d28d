"""bench.py's N > 1 plumbing on the CPU (gloo, --dry-run: a stub sealer in place of the engine):
`--gpus N` with no launcher starts the N rank processes itself (dist.launch_ranks) and rank 0 prints
one line whose n_gpus is the process group's world size; a launcher whose WORLD_SIZE disagrees with
--gpus ends the run with status 2; a failing rank's status reaches the caller."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    env.update(ATLS_NO_TORCH_RUNTIME="1", **kw)
    return env


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_launches_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["dry_run"] and d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 0 and d["scaling"] == "weak"


@pytest.mark.timeout(400)
def test_whole_c4_batch_exchange_from_rank0_at_8_ranks():
    """the sharded exchange (sharded_from_rank0) starts from the config's WHOLE batch on
    rank 0 -- C4's 1,048,576 records -- not rank 0's own shard; split 8 ways by bytes (131,072 each for
    C4's equal records), scattered, sealed by each rank (stub sealer on the CPU) and gathered back equal
    to rank 0 sealing the whole batch alone. Contents cut to 16 B per record so it fits a CPU run."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--dry-run", "--config", "c4_aes256gcm_1Mi_x_16KiB",
                        "--steps", "2", "--warmup", "1", "--dry-run-cap", "16"],
                       capture_output=True, text=True, timeout=360, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    sg = json.loads(lines[0])["sharded_from_rank0"]
    assert sg["records"] == 1048576 and sg["matches_single_gpu"] is True
    assert sg["records_per_rank"] == [131072] * 8


@pytest.mark.timeout(120)
def test_world_size_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=100, env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.timeout(240)
def test_failing_rank_status_reaches_caller():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--config", "no_such_config"],
                       capture_output=True, text=True, timeout=200, env=_env())
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.timeout(240)
@pytest.mark.parametrize("how", ["raise", "hang"])
def test_first_collective_failure_refuses_clearly(how):
    """if the process group's first collective fails (RCCL between distinct GPUs at init), the run
    refuses with status 4 and a message instead of hanging in its first barrier -- rank 1 raising there, and rank
    1 never answering (rank 0's watchdog fires after --comms-timeout)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1",
                        "--comms-timeout", "10"],
                       capture_output=True, text=True, timeout=200, env=_env(ATLS_TEST_COMMS_FAIL=how))
    assert r.returncode == 4, (r.returncode, r.stderr[-2000:])
    assert "failed at its first collective" in r.stderr, r.stderr[-2000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
