"""bench.py's one-line contract on a GPU (the fields the driver and the judge read): a short C2 run through the
HIP engine must print exactly one JSON line with the metric, a whole-job value, the HBM roofline object (achieved
/ peak = frac, the PMC traffic figure, the LDS-array fraction with its same-window clock), the open half with every
plaintext and status checked, and the CPU baseline of the oracle. Steps, settle times and the CPU sample are cut
short; the numbers are not asserted beyond being positive and self-consistent."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_bench_line_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--no-configs",
           "--sustain-s", "0.2", "--cpu-seconds", "0.5", "--cpu-threads", "4", "--settle-ms", "10",
           "--load-settle-ms", "20"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "open"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["dtype"] == "u8" and d["unit"] == "GiB/s" and d["vs_baseline"] is None
    assert d["config"]["workload"] == "c2_aes128gcm_64Ki_x_16KiB" and d["config"]["records_per_gpu"] == 65536
    assert d["value"] > 0 and d["ms_per_step"] > 0
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert rf["alg_bytes_per_launch"] == 65536 * (2 * 16385 + 16)
    assert rf["traffic"] is None or rf["traffic"] > rf["alg_bytes_per_launch"]
    lds = rf["lds"]
    assert lds["bound"] == "lds" and 0 < lds["frac"] < 1.2 and lds["sclk_MHz"] > 500
    assert "clock_in_window" in lds
    assert d["open"]["plaintext_and_status_ok"] is True and d["open"]["frac"] > 0
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["unit"] == "GiB/s" and cb["value"] > 0 and cb["cores"] >= 1 and cb["sample"]
