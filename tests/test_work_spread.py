"""The planned AES-GCM kernel's position mapping (gcm.hip gcm_kernel, ATLS_GCM_SPREAD): position p = wave *
grid + block of every row, odd rows reversed. Restated here: every work-list position is taken exactly once
for any grid / list size, and on the C5 shard's AES-GCM records (longest first, 1 KiB classes) the busiest
workgroup's load falls from ~1.18x to ~1.01x the mean. CPU only."""
import numpy as np
import pytest


def positions(cnt, grid, waves, spread=True):
    stride = grid * waves
    out = {}
    for b in range(grid):
        for w in range(waves):
            p = w * grid + b if spread else b * waves + w
            row = 0
            while row * stride < cnt:
                q = row * stride + (stride - 1 - p if spread and row & 1 else p)
                if q < cnt:
                    out.setdefault((b, w), []).append(q)
                row += 1
    return out


@pytest.mark.parametrize("cnt,grid", [(0, 4), (1, 256), (7, 3), (100, 8), (3073, 256), (16568, 256), (999, 17)])
def test_every_position_once(cnt, grid):
    got = sorted(q for qs in positions(cnt, grid, 12).values() for q in qs)
    assert got == list(range(cnt))
    if cnt:
        assert positions(cnt, grid, 12)[(0, 0)][0] == 0  # the single call's record: block 0, wave 0


def test_c5_balance():
    from anothertls_amd import workload

    b = workload.shard_batch("c5_mixed_256Ki_x_64B-16KiB", 0)
    suite = b["keys"]["suite"][b["recs"]["key_slot"]]
    ln = b["recs"]["len"][suite != 0x1303].astype(np.int64)
    order = np.argsort(-np.minimum(ln >> 10, 15), kind="stable")  # plan.hip: longest class first
    cost = ((ln + 1) // 16 + 4 + 63) // 64 + 3.0  # steps + per-record overhead (step-equivalents)
    cost = cost[order]
    load = {}
    for spread in (False, True):
        per_wg = np.zeros(256)
        for (blk, _), qs in positions(len(cost), 256, 12, spread).items():
            per_wg[blk] += cost[qs].sum()
        load[spread] = per_wg.max() / per_wg.mean()
    assert load[False] > 1.1 and load[True] < 1.03, load
