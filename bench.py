"""Benchmark: device-resident TLS-record AEAD throughput (BASELINE.json metric) on MI355X.

python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2_aes128gcm_64Ki_x_16KiB]
(--config c1_server_https_loopback_1MiB: BASELINE config C1, one connection's loopback through the native
batched socket path (atls_sb_*), MB/s, the Python mirror beside it and 64 / 256 connections under at_scale, with
the reference's per-record CPU path as cpu_baseline)
For N > 1 the driver launches one rank per GPU with torch.distributed.run; each rank seals
its own pre-sharded, device-resident batch of the config (records are independent, so there
is no data-path collective: weak scaling). One step = one atls_seal_batch over the whole
batch. Rank 0 prints one JSON line. `--gpus N` without a launcher (no WORLD_SIZE) starts the N
rank processes itself before anything touches the GPU; a launcher whose WORLD_SIZE differs from
--gpus, or a LOCAL_RANK without a GPU, ends the run with status 2. n_gpus is the world size the
process group reports. If the process group's first collective (RCCL's communicator between the GPUs)
fails or hangs, every rank exits with status 4 and says why on stderr, before anything is measured. A hung
post-timing exchange ends every rank with status 3 after rank 0 has printed the line.

Fields beyond the driver contract:
  roofline     — dominant kernel (AES-GCM seal): algorithmic bytes per launch (2L+16 per record:
                 read L, write L ciphertext + 16 tag) / average launch time from HIP events on
                 the engine's stream; peak 8 TB/s HBM3E; traffic = PMC-measured HBM bytes per
                 launch from profiles/ (null if not yet profiled); copy_GBps = a measured
                 device-to-device copy of the payload buffer (read + write) and frac_of_copy =
                 achieved / copy_GBps.
  wire_GiBps   — (--wire) the same records sealed as one contiguous wire stream, header || ct ||
                 tag per record (ATLS_MODE_WIRE), payload GiB/s from HIP events.
  open         — the decrypt half: open_batch over the sealed records of the same batch (GiB/s,
                 kernel_ms from HIP events, roofline frac with the same 2L+16 bytes per record),
                 statuses, lengths and (uniform configs) every plaintext byte checked; AES-GCM configs
                 add open.lds, the open kernels' LDS-array fraction at their own measured clock.
  cpu_baseline — the oracle (literal C restatement of the reference's algorithm: byte S-box
                 AES with bit-serial MixColumns, bit-serial GHASH) on a bounded sample of the
                 same records, on this host: --cpu-threads threads (value) and 1 thread
                 (value_1thread).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "GiB/s device-resident TLS-record AEAD (16 KiB recs); % HBM roofline @1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="c2_aes128gcm_64Ki_x_16KiB")
    p.add_argument("--records", type=int, default=None, help="override records per GPU")
    p.add_argument("--key-slots", type=int, default=None,
                   help="override the config's 4096 connections (= records: one key per record)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=16,
                   help="CPU-baseline threads (the GPU box's host share is 16 cores)")
    p.add_argument("--pcie", action="store_true", help="also time host-memory (PCIe-inclusive) batches")
    p.add_argument("--wire", action="store_true",
                   help="also time the same records sealed as one wire stream (ATLS_MODE_WIRE)")
    p.add_argument("--no-scatter", action="store_true",
                   help="N > 1: skip the sharded scatter / seal / gather of rank 0's batch")
    p.add_argument("--scatter-timeout", type=float, default=120.0,
                   help="N > 1: seconds the sharded exchange may take before the line is printed without it")
    p.add_argument("--no-open", action="store_true", help="skip the open (decrypt) half of the measurement")
    p.add_argument("--no-lazy-join", action="store_true",
                   help="join a mixed batch's side kernel at the end of every step (A/B of ATLS_FLAG_LAZY_JOIN)")
    p.add_argument("--no-configs", action="store_true",
                   help="skip the other BASELINE configs (C3, C4 shard, C5 shard) timed after the headline one")
    p.add_argument("--config-steps", type=int, default=10, help="timed steps of each of those configs")
    p.add_argument("--settle-ms", type=float, default=200.0,
                   help="before the warm-up steps, time the on-device copy rate for this long (it also brings the "
                        "GPU's clock up from idle, which a few 1-ms warm-up steps do not; 0 = after the steps)")
    p.add_argument("--load-settle-ms", type=float, default=300.0,
                   help="then run the config's own seals back to back for this long before the warm-up steps: the "
                        "clock under this load settles over ~100 ms (DESIGN §6), so the timed steps see the steady "
                        "state a serving engine runs at (untimed; 0 = off)")
    p.add_argument("--sustain-s", type=float, default=5.0,
                   help="after the timed steps, seal the headline batch back to back for this long (every rank) "
                        "and report the sustained rate (clocks under continuous load); 0 = skip")
    p.add_argument("--c1-threads", type=int, default=16, help="C1 at scale: worker threads per stream batch")
    p.add_argument("--dry-run-cap", type=int, default=64,
                   help="--dry-run: content bytes per record of the whole-batch exchange rehearsal")
    p.add_argument("--comms-timeout", type=float, default=180.0,
                   help="N > 1: seconds the process group's first collective (RCCL's communicator set-up) may take "
                        "before every rank exits with status 4")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU only (gloo): the launcher, rendezvous, timing and JSON line with a stub sealer "
                        "instead of the engine (tests of the N > 1 plumbing)")
    return p.parse_args()


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo), for cpu_baseline."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def _oracle_rate(ora, okeys, recs, inbuf_host, n_rec, threads, budget_s):
    """Oracle seal of records [0, n_rec) repeated until ~budget_s; returns (GiB/s, records, bytes, s)."""
    aux = np.zeros(16, np.uint8)
    out = np.zeros(int(recs["out_off"][n_rec - 1]) + 16400, np.uint8)
    tags = np.zeros(16 * n_rec, np.uint8)
    chunk = max(threads, 1) * (1 if threads == 1 else 16)
    done, payload, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        lo = done % n_rec
        sub = recs[lo:min(lo + chunk, n_rec)].copy()
        orecs = (ora.OraRec * len(sub)).from_buffer_copy(sub.tobytes())
        ora.seal_batch(okeys, orecs, inbuf_host, aux, out, tags, threads)
        payload += int(sub["len"].sum()) + len(sub)
        done += len(sub)
    dt = time.perf_counter() - t0
    return payload / dt / 2**30, done, payload, dt


def cpu_baseline(batch, inbuf_host, budget_s, threads):
    """The oracle (literal C restatement of the reference's AES-GCM: byte S-box rounds with
    bit-serial MixColumns, bit-serial GHASH) sealing the first records of this rank's batch on
    this host: `threads` threads (records split across pthreads) for ~budget_s, plus a
    1-thread run for ~budget_s / 4."""
    import oracle as ora

    keys, recs = batch["keys"], batch["recs"]
    okeys = (ora.OraKey * len(keys)).from_buffer_copy(keys.tobytes())
    n_rec = min(len(recs), 4096)
    v1, d1, p1, t1 = _oracle_rate(ora, okeys, recs, inbuf_host, n_rec, 1, budget_s / 4)
    vn, dn, pn, tn = _oracle_rate(ora, okeys, recs, inbuf_host, n_rec, threads, budget_s)
    return dict(value=vn, unit="GiB/s", cores=threads, cpu_model=cpu_model(), kind="port", value_1thread=v1,
                sample=f"{dn} record seals ({pn} B AEAD payload) cycling over the first {n_rec} records of the same "
                       f"batch, oracle/ref_restatement.c ora_seal_batch, {threads} threads, {tn:.1f} s; 1 thread: "
                       f"{d1} records ({p1} B) in {t1:.1f} s")


def whole_batch(args, world):
    """The config's WHOLE record batch (BASELINE's stated size: C4 1 Mi records, C5 256 Ki, C2 / C3 64 Ki),
    or --records x world records when --records overrides the per-GPU count."""
    from anothertls_amd import workload

    n = args.records * world if args.records else None
    return workload.config_batch(args.config, n=n, n_keys=args.key_slots)


def sharded_exchange(batch, seal, make_input, zeros, sync, device=None, reps=3):
    """A batch that arrives whole at rank 0 (C4 is stated as 1 Mi records sharded across 8
    GPUs) sealed by every rank through dist.seal_sharded: byte-balanced split (atls_partition), RCCL
    point-to-point scatter of the input and output ranges, each rank's engine on its range, gather of
    the sealed ranges and tags back. Rank 0 first seals the whole batch alone, the reference the
    gathered bytes must equal. Returns (rank 0) GiB/s of AEAD payload for scatter + seal + gather,
    max time over ranks; None on the other ranks."""
    from anothertls_amd import dist

    recs = batch["recs"]
    n = len(recs)
    rank = dist.env_ranks()[0]
    inp = out = tags = ref_out = ref_tags = None
    if rank == 0:
        inp = make_input(batch["in_bytes"] + 16)
        ref_out, ref_tags = zeros(batch["out_bytes"] + 16), zeros(16 * n)
        seal(recs, inp, ref_out, ref_tags)  # the whole batch on rank 0's GPU alone
        out, tags = zeros(batch["out_bytes"] + 16), zeros(16 * n)
    sync()

    def run():
        dist.seal_sharded(seal, recs, inp, out, tags, device=device)

    run()  # warm-up: communicators, staging
    wall = dist.timed_steps(run, reps, 0, sync, device)
    if rank != 0:
        return None
    import torch

    match = bool(torch.equal(out, ref_out) and torch.equal(tags, ref_tags))
    world = dist.world_size()
    import anothertls_amd as atls

    first = atls.partition(recs, world)
    return {"GiBps": round(batch["payload"] * reps / wall / 2**30, 3), "ms": round(wall / reps * 1e3, 3),
            "matches_single_gpu": match, "records": n, "payload_bytes": batch["payload"],
            "records_per_rank": [int(first[r + 1] - first[r]) for r in range(world)],
            "path": "rank 0 holds the whole batch; dist.seal_sharded: atls_partition byte split, torch.distributed "
                    "P2P (RCCL over xGMI) scatter / gather, every rank's engine on its range"}


C1 = "c1_server_https_loopback_1MiB"


def c1_cpu_reference(body, reps):
    """BASELINE config C1's reference path: the oracle's restatement of RecordPayloadProtection
    (ora_record_seal / ora_record_open, one record per call as tls_write / tls_read do) through
    the same 127.0.0.1 socket loop as the GPU run (tools/c1_loopback.py). Returns seconds."""
    import oracle as ora

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import c1_loopback as c1

    rc, key, iv = ora.key_from_secret(32, c1.SECRET, 16, 12)
    assert rc == 0
    frags = [body[i * c1.CONTENT:(i + 1) * c1.CONTENT] for i in range(c1.N_REC)]

    def seal_body():
        parts = []
        for seq, f in enumerate(frags):
            rc, wire = ora.record_seal(0x1301, key, iv, seq, 23, f)
            assert rc == 0
            parts.append(wire)
        return b"".join(parts)

    def open_wire(wire):
        pt, pos = [], 0
        for seq in range(c1.N_REC):
            n = (wire[pos + 3] << 8) | wire[pos + 4]
            rc, frag, ctype = ora.record_open(0x1301, key, iv, seq, wire[pos:pos + 5 + n])
            assert rc == 0 and ctype == 23
            pt.append(frag)
            pos += 5 + n
        return b"".join(pt)

    dt, pt = c1._loop(seal_body, open_wire, c1.N_REC * (5 + c1.CONTENT + 1 + 16), reps)
    assert pt == body
    return dt


def run_c1(args):
    """C1 (server_https over loopback, 1 MiB body of 64 x 16 KiB AES-128-GCM records, one connection): the
    native batched socket path (tools/c1_loopback_native, atls_sb_*: one WIRE seal batch per body, one open batch
    per receive round, every byte checked) is `value`; the Python mirror (tools/c1_loopback.py run_gpu,
    anothertls_amd.stream.StreamBatch) beside it; the reference's per-record CPU path over the same loop is the
    cpu_baseline. K steps = K bodies; the native tool warms up with K bodies first (its page-locked arenas at
    their size). The native runs go first, before this process opens engines of its own: a second process's
    hardware queues on the same GPU doubled the tool's flush time (1 MiB flushes are launch-latency bound)."""
    import subprocess

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import c1_loopback as c1

    exe = os.path.join(ROOT, "tools", "c1_loopback_native")

    def native_run(reps, conns, threads):
        out = subprocess.run([exe, str(reps), str(conns), str(threads)], capture_output=True, text=True, timeout=300)
        if out.returncode != 0 or not out.stdout.strip():
            return {"error": out.stderr[-300:]}
        line = json.loads(out.stdout.strip().splitlines()[-1])
        line.pop("config", None)
        return line

    native, scale = None, []
    if os.path.exists(exe):
        native = native_run(args.steps, 1, 1)
        if not native.get("verified"):
            raise RuntimeError(f"c1_loopback_native: {native}")
        # C1 at scale: 64 and 256 connections with worker threads; the server and client sides
        # run in one process, so T threads per side is 2T on the host's CPU share (16 on the GPU box)
        for conns, reps in ((64, 16), (256, 4)):
            for threads in sorted({1, 8, args.c1_threads}):
                scale.append(native_run(reps, conns, threads))
    body = np.random.default_rng(0xC1).integers(0, 256, c1.N_REC * c1.CONTENT, dtype=np.uint8).tobytes()
    dt, pt = c1.run_gpu(body, args.steps)
    assert pt == body
    py = {"MBps": round(args.steps * len(body) / dt / 1e6, 1), "ms_per_step": round(dt / args.steps * 1e3, 3),
          "warmup": 1, "path": "anothertls_amd.stream.StreamBatch (WIRE mode), Python"}
    if native:
        value, ms, warm = native["gpu_MBps"], native["phase_ms"]["wall"] / args.steps, args.steps
        path = "native atls_stream_batch (include/atls.h atls_sb_*, WIRE mode), one connection, every byte checked"
    else:  # the tool is built by __graft_entry__.build(); without it the Python mirror's rate is the value
        value, ms, warm, path = py["MBps"], py["ms_per_step"], 1, py["path"]
    result = {"metric": "MB/s of response body through seal -> 127.0.0.1 socket -> open (server_https loopback)",
              "value": value, "unit": "MB/s", "n_gpus": 1,
              "steps": args.steps, "warmup": warm, "ms_per_step": round(ms, 3),
              "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "u8",
              "data": "synthetic 1 MiB body, RFC 8448 server traffic secret",
              "config": {"workload": C1, "records_per_body": c1.N_REC, "record_content": c1.CONTENT,
                         "suite": "TLS_AES_128_GCM_SHA256", "connections": 1, "path": path},
              "python_StreamBatch": py}
    if native:
        result["native_phase_ms"] = native["phase_ms"]
        result["at_scale"] = {"runs": scale, "unit": "MB/s of response body, seal -> 127.0.0.1 TCP -> open, every byte checked",
                              "path": "native atls_stream_batch: a flush seals its records in engine batches of <= 64 MiB "
                                      "while the previous batch is sent, a receive round opens in such batches; "
                                      "T worker threads per batch (atls_sb_set_threads); the server writes the "
                                      "next body while the last is flushed"}
    if not args.no_cpu_baseline:
        t = c1_cpu_reference(body, 1)
        result["cpu_baseline"] = {"value": round(len(body) / t / 1e6, 3), "unit": "MB/s", "cores": 1,
                                  "cpu_model": cpu_model(), "kind": "port",
                                  "sample": "one 1 MiB body (64 records) through the same socket loop, oracle "
                                            "ora_record_seal / ora_record_open per record"}
    print(json.dumps(result), flush=True)


def _stub_sealer():
    """--dry-run's stand-in for the engine on CPU tensors: content XOR 0x5A and the content type out,
    tag = (seq, len) -- deterministic per record whatever the offsets, so a sharded seal must equal the
    whole batch's."""

    def seal(recs, inp, out, tags):
        L = recs["len"].astype(np.int64)
        tot = int(L.sum())
        a, o = inp.numpy(), out.numpy()
        if tot:
            start = np.repeat(np.cumsum(L) - L, L)
            j = np.arange(tot, dtype=np.int64) - start
            o[np.repeat(recs["out_off"].astype(np.int64), L) + j] = a[np.repeat(recs["in_off"].astype(np.int64), L) + j] ^ 0x5A
        o[recs["out_off"].astype(np.int64) + L] = recs["content_type"]
        t = np.zeros((len(recs), 2), np.uint64)
        t[:, 0], t[:, 1] = recs["seq"], recs["len"]
        tags.numpy()[:] = t.view(np.uint8).ravel()

    return seal


def run_dry(args):
    """--dry-run: this rank's part of an N-rank job on the CPU (gloo) with a stub sealer (a byte XOR
    over a small C2-shaped shard) in place of the engine -- the launcher, rendezvous, barrier +
    max-over-ranks timing and the JSON line of the real run, without a GPU (tests/test_bench_launch.py).
    For N > 1 also the whole-batch exchange of the real run (sharded_from_rank0) over the config's full
    record list -- every record, slot and sequence number, contents cut to --dry-run-cap bytes so C4's
    1 Mi records fit a CPU rehearsal."""
    from anothertls_amd import dist, workload

    rank, _, world = dist.env_ranks()
    dist.init("gloo")
    dist.check_comms(None, args.comms_timeout, "gloo")
    batch = workload.shard_batch(args.config, rank, n=args.records or 64)
    buf = np.random.default_rng(rank).integers(0, 256, batch["in_bytes"], dtype=np.uint8)
    out = np.empty_like(buf)

    def step():
        np.bitwise_xor(buf, 0x5A, out=out)

    wall = dist.timed_steps(step, args.steps, args.warmup, lambda: None)
    ranks = dist.world_size()
    line = {"metric": METRIC, "value": round(dist.whole_job_rate(batch["payload"], args.steps, wall, ranks), 3),
            "unit": "GiB/s", "n_gpus": ranks, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "dry_run": True, "config": {"workload": args.config, "records_per_gpu": len(batch["recs"])}}
    if ranks > 1 and not args.no_scatter:
        import torch

        whole = workload.capped(whole_batch(args, ranks), args.dry_run_cap)
        sg = sharded_exchange(
            whole, _stub_sealer(),
            lambda nb: torch.from_numpy(np.random.default_rng(5).integers(0, 256, nb, dtype=np.uint8)),
            lambda nb: torch.zeros(nb, dtype=torch.uint8), lambda: None, reps=1)
        if rank == 0:
            sg["dry_run_content_cap"] = args.dry_run_cap
            line["sharded_from_rank0"] = sg
    if rank == 0:
        print(json.dumps(line), flush=True)
    dist.close()


def open_descs(recs):
    """Open descriptors for the sealed records of a TLS-mode batch: each reads its ciphertext
    (content || type, len + 1 bytes) at the seal's out_off and writes the inner plaintext back to
    the same offset of a separate buffer (RecordPayloadProtection::decrypt, record.rs:201-240)."""
    o = recs.copy()
    o["in_off"] = recs["out_off"]
    o["len"] = recs["len"] + 1
    return o


# The BASELINE configs timed beside the headline one: C3 whole, the per-GPU shards of C4
# and C5 (1/8 of their 8-GPU batches; at N GPUs every rank runs its own shard, so at N = 8 they are the
# whole configs).
EXTRA_CONFIGS = ("c3_chacha20poly1305_64Ki_x_1.5KiB", "c4_aes256gcm_1Mi_x_16KiB", "c5_mixed_256Ki_x_64B-16KiB")


def copy_probe(d_in, d_out, min_ms):
    """On-device copy rate (read + write GB/s) of this batch's buffers, d_in -> d_out, repeated for at
    least min_ms of GPU time. Run before the warm-up steps it also takes the GPU out of its idle clock
    state: MI355X's clock ramps over ~25 ms of load, longer than a few warm-up steps."""
    nbytes = min(d_in.numel(), d_out.numel())
    src, dst = d_in[:nbytes], d_out[:nbytes]
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dst.copy_(src)
    torch.cuda.synchronize()
    reps, total_ms = 0, 0.0
    c0.record()
    while True:
        for _ in range(10):
            dst.copy_(src)
        reps += 10
        c1.record()
        c1.synchronize()
        total_ms = c0.elapsed_time(c1)
        if total_ms >= min_ms:
            break
    return 2 * nbytes * reps / (total_ms * 1e-3) / 1e9


# LDS-array roofline of the AES-GCM record kernels. The static instruction mix per 16-byte
# block: AES-CTR by two-table T-table rounds with counter-mode caching -- 1 + 4 + 16 x (NR - 2) conflict-free
# ds_read_b32 (133 for AES-128, 165 for AES-192, 197 for AES-256) -- and one GHASH product by the 4-bit table,
# 32 ds_read_b128. A wave-instruction serves 64 blocks and costs 2 (b32) / 4 (b128) LDS-array cycles
# (MI355X_MICROARCH.md §LDS table). A record of AEAD length L has ceil(L/16) + 1 AES blocks (its counter
# blocks and E_K(J0)) and ceil(L/16) + 2 GHASH products (one AAD block, the ciphertext, the length block).
LDS_B32_PER_AES_BLOCK = {10: 133, 12: 165, 14: 197}
LDS_CYCLES_B32, LDS_CYCLES_B128, GHASH_B128_PER_BLOCK = 2, 4, 32


def lds_cycles_per_launch(batch):
    """Algorithmic LDS-array CU-cycles of one seal launch over an AES-GCM batch (None unless every record is
    AES-GCM: a mixed batch's launch interval also holds the VALU-bound ChaCha20-Poly1305 kernel): the
    per-block static mix above times the blocks; table builds, lane combines and the lanes idle in a record's
    last step are not counted (the measured SQ_LDS_IDX_ACTIVE includes them)."""
    keys, recs = batch["keys"], batch["recs"]
    suite = keys["suite"][recs["key_slot"]]
    aes = suite != 0x1303
    if not aes.all():
        return None
    L = recs["len"][aes].astype(np.int64) + 1  # TLS: content || type
    nr = np.where(keys["key_len"][recs["key_slot"][aes]] == 16, 10, np.where(keys["key_len"][recs["key_slot"][aes]] == 24, 12, 14))
    b32 = np.vectorize(LDS_B32_PER_AES_BLOCK.get)(nr)
    blocks = (L + 15) // 16
    cyc = (blocks + 1) * b32 * LDS_CYCLES_B32 + (blocks + 2) * GHASH_B128_PER_BLOCK * LDS_CYCLES_B128
    return float(cyc.sum()) / 64.0


class ClockProbe:
    """The shader clock over a timed window, from the same launches as the kernel time it is paired with
    (a clock read in a separate pass after a synchronize had dropped and inflated lds.frac). The
    probe (atls_clock_probe, 16 one-wave workgroups on a second stream, no LDS) is enqueued as the window's
    first launch is, sleeps through the first 15 % of the window's expected span and reads s_memtime against
    s_memrealtime over the next 70 %; `mhz()` (after the window's synchronize) is the median over the waves."""

    WGS = 16
    _made = {}

    @classmethod
    def of(cls, eng, dev):
        """One probe (and one side stream) per engine for the whole run. A fresh torch stream per config can land on
        the engine stream's hardware queue (4 per process, handed out in turn as streams are created): the probe
        then runs in that queue's order, before the seals, on an idle GPU -- round 6's first C4 whole-batch leg read
        2,396 MHz and its timed wall grew by the probe's span. The stream made with the first config's probe
        (after the engine's) is one the seals do not queue behind; `overlap` checks it every window."""
        key = (id(eng), str(dev))
        if key not in cls._made:
            cls._made[key] = cls(eng, dev)
        return cls._made[key]

    def __init__(self, eng, dev):
        self.eng, self.dev = eng, dev
        self.side = torch.cuda.Stream(device=dev)
        self.out = torch.zeros(2 * self.WGS, dtype=torch.int64, device=dev)
        self.p0, self.p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # one probe launch here, before any timed window: the first launch of a kernel loads its code object
        # (milliseconds with the host blocked and the GPU idle), which inside the window left the GPU idle and
        # its clock falling (profiles/r06/first/: C2's window at 1.93 GHz and 1.12 ms per launch)
        self.eng.clock_probe(self.out, wgs=self.WGS, delay_us=0, spin_us=1, stream=self.side.cuda_stream)
        torch.cuda.synchronize(dev)

    def start(self, n_launch, est_ms):
        span_us = n_launch * est_ms * 1e3
        self.p0.record(self.side)
        self.eng.clock_probe(self.out, wgs=self.WGS, delay_us=int(0.15 * span_us), spin_us=max(20, int(0.7 * span_us)),
                             stream=self.side.cuda_stream)
        self.p1.record(self.side)

    def mhz(self):
        torch.cuda.synchronize(self.dev)
        o = self.out.cpu().numpy().reshape(self.WGS, 2).astype(np.float64)
        return float(np.median(100.0 * o[:, 0] / np.maximum(o[:, 1], 1)))

    def overlap(self, w0, w1):
        """Whether the probe ran inside the window [w0, w1] (HIP events on the engine stream): its end no later
        than the window's end (+2 %). A probe that could not be placed beside the window's launches reads the
        clock after them, which is not theirs; the line then says so (clock_in_window false)."""
        torch.cuda.synchronize(self.dev)
        win = w0.elapsed_time(w1)
        end = w0.elapsed_time(self.p1)
        return {"window_ms": round(win, 3), "probe_end_ms": round(end, 3), "in_window": bool(end <= 1.02 * win + 0.05)}


def settle(launch, sync, ms):
    """Run `launch` back to back, untimed, for `ms` milliseconds (synchronising every 8 launches): the clock under
    this load settles over ~100 ms. Returns the mean host ms per launch (an estimate of the launch's
    span, for the clock probe's timing), or None when ms <= 0."""
    if ms <= 0:
        return None
    count, t0 = 0, time.perf_counter()
    t_end = t0 + ms * 1e-3
    while time.perf_counter() < t_end:
        for _ in range(8):
            launch()
        sync()
        count += 8
    return (time.perf_counter() - t0) * 1e3 / count


def launch_ms(launch, stream, sync, n=3):
    """The mean launch time of n launches from HIP events (the clock probe's span estimate without a settle)."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(n):
        launch()
    e1.record(stream)
    sync()
    return e0.elapsed_time(e1) / n


def lds_roofline(batch, kern_ms, sclk_mhz, cus):
    """roofline.lds: the launch's algorithmic LDS-array cycles at the measured clock on every CU, as a
    fraction of the measured launch time."""
    cyc = lds_cycles_per_launch(batch)
    if cyc is None or not sclk_mhz:
        return None
    t_ms = cyc / cus / (sclk_mhz * 1e3)
    return {"bound": "lds", "cycles_per_launch": round(cyc), "sclk_MHz": round(sclk_mhz, 1), "cus": cus,
            "t_min_ms": round(t_ms, 4), "kernel_ms": round(kern_ms, 4), "frac": round(t_ms / kern_ms, 4),
            "per_block": "AES-CTR 1+4+16(NR-2) ds_read_b32 x 2 cyc + GHASH 32 ds_read_b128 x 4 cyc, per 64 blocks",
            "clock": "atls_clock_probe beside the timed launches themselves, enqueued with the first of them (s_memtime / "
                     "s_memrealtime over the middle 70 % of the window, median of 16 waves)"}


def measure(name, eng, dev, rank, world, steps, warmup, lazy, records=None, key_slots=None, keep=False,
            settle_ms=0.0, load_settle_ms=0.0, do_open=True):
    """This rank's shard of config `name`, device-resident: `steps` timed seals (barrier + sync on both
    sides, max over ranks) with the kernels' interval from HIP events on the engine stream, then as many
    opens of the sealed records with every status, length and (uniform configs) plaintext byte checked.
    settle_ms > 0: the copy probe (copy_probe) runs that long first. Returns the numbers (and with
    keep=True the batch and its device buffers)."""
    import anothertls_amd as atls
    from anothertls_amd import dist, workload

    batch = workload.shard_batch(name, rank, n=records, n_keys=key_slots)
    recs = batch["recs"]
    n = len(recs)
    eng.set_keys(batch["keys"])
    g = torch.Generator(device=dev).manual_seed(workload.SEEDS["payload"] + rank)
    d_in = torch.randint(0, 256, (batch["in_bytes"],), dtype=torch.uint8, device=dev, generator=g)
    d_out = torch.empty(batch["out_bytes"], dtype=torch.uint8, device=dev)
    d_tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    d_recs = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
    torch.cuda.synchronize(dev)
    copy_gbps = copy_probe(d_in, d_out, settle_ms) if settle_ms > 0 else None
    # LAZY_JOIN: a mixed batch's ChaCha20-Poly1305 kernel is not joined back at the end of each step,
    # so the next step's plan and AES-GCM kernel start beside it (C5); no effect on one-suite batches
    flags = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS | atls.FLAG_NO_SYNC | (atls.FLAG_LAZY_JOIN if lazy else 0)
    stream = torch.cuda.ExternalStream(eng.stream, device=dev)
    # raw device pointers: the buffers are resident and synchronized above, so no per-step wait
    # on torch's stream is needed (Engine._after_torch)
    p_recs, p_in, p_aux, p_out, p_tags = (t.data_ptr() for t in (d_recs, d_in, d_aux, d_out, d_tags))

    def sync():
        eng.sync()
        torch.cuda.synchronize(dev)

    def seal_launch():
        eng.seal_batch(p_recs, p_in, p_aux, p_out, p_tags, flags=flags, n=n)

    # the same seals back to back, untimed, until the clock has settled under this load: a C2 launch takes
    # 1.29-1.46 ms for the first few after other work, ~1.0 ms after ~100 ms
    lds_kind = lds_cycles_per_launch(batch) is not None
    probe = ClockProbe.of(eng, dev) if lds_kind else None
    est_ms = settle(seal_launch, sync, load_settle_ms) or launch_ms(seal_launch, stream, sync)

    # kernel time of the same steps from HIP events on the engine's stream; the clock probe beside them
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    marks = {"n": 0}

    def timed_step():
        if marks["n"] == warmup:
            eng.join()  # the interval holds exactly the timed steps' kernels
            if probe:
                probe.start(steps, est_ms)
            ev0.record(stream)
        seal_launch()
        marks["n"] += 1
        if marks["n"] == warmup + steps:
            eng.join()
            ev1.record(stream)

    def step_sync():
        # the engine's streams and torch's current stream, not the probe's side stream: the wall clock of the
        # timed steps never waits for the probe (were it placed late, it would otherwise stretch the window)
        eng.sync()
        torch.cuda.current_stream(dev).synchronize()

    wall = dist.timed_steps(timed_step, steps, warmup, step_sync, dev)
    sync()
    kern_ms = ev0.elapsed_time(ev1) / steps
    payload = batch["payload"]  # sum of AEAD lengths (content + type byte)
    alg_bytes = 2 * payload + 16 * n
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    m = {"batch": batch, "n": n, "wall": wall, "kern_ms": kern_ms, "payload": payload, "alg_bytes": alg_bytes,
         "achieved": achieved, "value": dist.whole_job_rate(payload, steps, wall, world), "flags": flags,
         "stream": stream, "sync": sync, "copy_gbps": copy_gbps}
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    if probe:
        # the LDS roofline is in cycles: the clock of the timed launches themselves
        m["sclk_mhz"] = probe.mhz()
        m["lds"] = lds_roofline(batch, kern_ms, m["sclk_mhz"], cus)
        if m["lds"]:
            m["lds"]["clock_in_window"] = probe.overlap(ev0, ev1)

    if do_open:
        # ---- the decrypt half (Gcm::decrypt, gcm.rs:142-157, via record.rs:201-240) over the records
        # just sealed: same records, same bytes per record (read L + 16-byte tag, write L) ----
        orecs = open_descs(recs)
        d_orecs = torch.from_numpy(orecs.view(np.uint8).copy()).to(dev)
        d_pt = torch.zeros(batch["out_bytes"], dtype=torch.uint8, device=dev)
        d_res = torch.zeros(8 * n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        q_recs, q_pt, q_res = d_orecs.data_ptr(), d_pt.data_ptr(), d_res.data_ptr()

        def open_launch():
            eng.open_batch(q_recs, p_out, p_aux, p_tags, q_pt, q_res, flags=flags, n=n)

        # the opens' own load settle, as the seals': after the seal leg's host work the clock has dropped, and
        # a few warm-up opens do not bring it back (tools/open_order_probe.py: opens and seals alternated in
        # blocks of 20 run within 1-2 % of each other, C2 1.005-1.024 vs 0.999-1.017 ms)
        est_open = settle(open_launch, sync, load_settle_ms) or launch_ms(open_launch, stream, sync)
        o0, o1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i in range(warmup + steps):
            if i == warmup:
                eng.join()
                if probe:
                    probe.start(steps, est_open)
                o0.record(stream)
            open_launch()
        eng.join()
        o1.record(stream)
        sync()
        open_ms = o0.elapsed_time(o1) / steps
        res = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
        ok = bool((res["status"] == 0).all() and (res["content_len"] == recs["len"]).all()
                  and (res["content_type"] == 23).all())
        lens = recs["len"]
        if ok and n > 1 and (lens == lens[0]).all() and (np.diff(recs["in_off"]) == recs["in_off"][1] - recs["in_off"][0]).all() \
                and (np.diff(recs["out_off"]) == recs["out_off"][1] - recs["out_off"][0]).all():
            # uniform records (C2-C4): every plaintext byte of every record against the sealed input
            L, si, so = int(lens[0]), int(recs["in_off"][1] - recs["in_off"][0]), int(recs["out_off"][1] - recs["out_off"][0])
            ok = bool(torch.equal(d_pt[: n * so].view(n, so)[:, :L], d_in[: n * si].view(n, si)[:, :L]))
        open_ach = alg_bytes / (open_ms * 1e-3) / 1e9  # read L+1 ciphertext + 16 tag, write L+1 plaintext
        m["open"] = {"GiBps": round(payload / (open_ms * 1e-3) / 2**30, 3), "kernel_ms": round(open_ms, 4),
                     "achieved_GBps": round(open_ach, 1), "frac": round(open_ach / HBM_PEAK_GBPS, 4),
                     "plaintext_and_status_ok": ok,
                     "what": "open_batch over the sealed records (device-resident, same batch), HIP events on the "
                             "engine stream over the timed steps"}
        if probe:
            # the open kernels' LDS-array fraction at the clock of the timed opens themselves
            ol = lds_roofline(batch, open_ms, probe.mhz(), cus)
            if ol:
                m["open"]["lds"] = {"sclk_MHz": ol["sclk_MHz"], "t_min_ms": ol["t_min_ms"], "frac": ol["frac"],
                                    "clock_in_window": probe.overlap(o0, o1)["in_window"]}
        del d_orecs, d_pt, d_res
    if keep:
        m.update(d_in=d_in, d_out=d_out, d_tags=d_tags, d_aux=d_aux, d_recs=d_recs)
    else:
        del d_in, d_out, d_tags, d_recs
        torch.cuda.empty_cache()
    return m


def config_summary(name, m, steps):
    """One `configs` entry: seal and open GiB/s, kernel interval and HBM-roofline fraction."""
    from anothertls_amd import workload

    suite, _, clen = workload.CONFIGS[name]
    return {"records_per_gpu": m["n"], "steps": steps, "GiBps": round(m["value"], 3),
            "kernel_ms": round(m["kern_ms"], 4), "achieved_GBps": round(m["achieved"], 1),
            "frac": round(m["achieved"] / HBM_PEAK_GBPS, 4), "alg_bytes_per_launch": m["alg_bytes"],
            "suite": suite if isinstance(suite, str) else suite.name,
            "aead_bytes_per_record": (clen + 1) if isinstance(clen, int) else "content U{64..16384}+1",
            "open": {k: v for k, v in m["open"].items() if k != "what"},
            **({"lds": {k: v for k, v in m["lds"].items() if k not in ("per_block", "clock")}} if m.get("lds") else {})}


def main():
    args = parse()
    if args.config == C1:
        return run_c1(args)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # --gpus N without a launcher: one fresh process per GPU, as torch.distributed.run would start
        # them; this process has not touched the GPU (nor loaded the engine) and only waits for them
        from anothertls_amd import dist

        sys.exit(dist.launch_ranks([os.path.abspath(__file__), *sys.argv[1:]], args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} from the launcher but --gpus {args.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)
    if args.dry_run:
        return run_dry(args)
    from anothertls_amd import dist

    rank, local, world = dist.env_ranks()
    ndev = torch.cuda.device_count()  # does not initialise the GPU
    if local >= ndev:
        print(f"bench.py: LOCAL_RANK {local} but {ndev} visible GPU(s)", file=sys.stderr, flush=True)
        sys.exit(2)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init("nccl", dev)
    # the first collective builds RCCL's communicator between the GPUs: a failure or a hang there ends every rank
    # with status 4 and a message, before anything is measured
    dist.check_comms(dev, args.comms_timeout)
    world = dist.world_size()  # as the process group reports it

    import anothertls_amd as atls
    from anothertls_amd import workload

    eng = atls.Engine(local)
    # this rank's shard of the config's record stream (weak scaling: fixed records per GPU)
    m = measure(args.config, eng, dev, rank, world, args.steps, args.warmup, not args.no_lazy_join,
                records=args.records, key_slots=args.key_slots, keep=True, settle_ms=args.settle_ms,
                load_settle_ms=args.load_settle_ms, do_open=not args.no_open)
    batch, recs, n, payload = m["batch"], m["batch"]["recs"], m["n"], m["payload"]
    d_in, d_out, d_tags, d_aux = m["d_in"], m["d_out"], m["d_tags"], m["d_aux"]
    flags, stream, sync, kern_ms, achieved, alg_bytes = m["flags"], m["stream"], m["sync"], m["kern_ms"], m["achieved"], m["alg_bytes"]

    # measured on-device copy bandwidth: read + write of this batch's payload buffer, from the
    # probe before the warm-up steps (or here, with --settle-ms 0)
    copy_gbps = m["copy_gbps"] or copy_probe(d_in, d_out, 5.0)

    # sustained rate: the same seal launched back to back for --sustain-s seconds on every rank (the clock
    # under continuous load; outside the timed region above, which stays the reported value)
    sustained = None
    if args.sustain_s > 0:
        n_sus = max(1, int(args.sustain_s * 1e3 / max(kern_ms, 1e-3)))
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        p_recs, p_in, p_aux, p_out, p_tags = (t.data_ptr() for t in (m["d_recs"], d_in, d_aux, d_out, d_tags))
        probe = torch.zeros(32, dtype=torch.int64, device=dev)
        side = torch.cuda.Stream(device=dev)
        eng.join()
        sync()
        span_us = n_sus * kern_ms * 1e3  # the probe reads the clock over the middle of the leg
        eng.clock_probe(probe, wgs=16, delay_us=int(0.3 * span_us), spin_us=int(0.4 * span_us), stream=side.cuda_stream)
        s0.record(stream)
        for _ in range(n_sus):
            eng.seal_batch(p_recs, p_in, p_aux, p_out, p_tags, flags=flags, n=n)
        eng.join()
        s1.record(stream)
        sync()
        sus_ms = s0.elapsed_time(s1) / n_sus
        o = probe.cpu().numpy().reshape(16, 2).astype(np.float64)
        sus_sclk = float(np.median(100.0 * o[:, 0] / np.maximum(o[:, 1], 1)))
        sus_ach = alg_bytes / (sus_ms * 1e-3) / 1e9
        sustained = {"seconds": round(sus_ms * n_sus / 1e3, 2), "launches": n_sus, "kernel_ms": round(sus_ms, 4),
                     "GiBps_per_gpu": round(payload / (sus_ms * 1e-3) / 2**30, 3),
                     "frac": round(sus_ach / HBM_PEAK_GBPS, 4), "sclk_MHz": round(sus_sclk, 1),
                     "what": "rank 0's seals back to back after the timed steps (HIP events); not the reported value"}
        lds_sus = lds_roofline(batch, sus_ms, sus_sclk, torch.cuda.get_device_properties(dev).multi_processor_count)
        if lds_sus:
            sustained["lds_frac"] = lds_sus["frac"]

    result = None
    if rank == 0:
        traffic = None
        tf = os.path.join(ROOT, "profiles", "traffic.json")
        if os.path.exists(tf):
            t = json.load(open(tf)).get(args.config)
            traffic = t.get("hbm_bytes_per_launch") if t else None
        suite, _, clen = workload.CONFIGS[args.config]
        result = {
            "metric": METRIC,
            "value": round(m["value"], 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(m["wall"] / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (device torch.randint payload, seeded keys/IVs)",
            "config": {"workload": args.config, "records_per_gpu": n,
                       "aead_bytes_per_record": (clen + 1) if isinstance(clen, int) else "content U{64..16384}+1",
                       "suite": suite if isinstance(suite, str) else suite.name, "key_slots": len(batch["keys"]),
                       "mode": "TLS (inner type byte, AAD header, per-record nonce derived on device)",
                       "parallelism": f"records sharded per GPU, dp{world}, no data-path collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": alg_bytes,
                         "copy_GBps": round(copy_gbps, 1), "frac_of_copy": round(achieved / copy_gbps, 4),
                         "lds": m.get("lds")},
        }
        if "open" in m:
            result["open"] = m["open"]
        if sustained:
            result["sustained"] = sustained
        if world == 1 and not args.no_cpu_baseline:
            sample = min(n, 4096)
            h_in = d_in[: int(recs["in_off"][sample - 1]) + int(recs["len"][sample - 1]) + 16].cpu().numpy()
            result["cpu_baseline"] = cpu_baseline(batch, h_in, args.cpu_seconds, args.cpu_threads)
        if args.pcie and world == 1:
            # host-memory batches (the socket path): the engine stages them over PCIe; pinned
            # (page-locked) host buffers as a record layer would keep its socket buffers in
            def pinned(nbytes):
                return torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).numpy()

            h_in, h_out, h_tags = pinned(batch["in_bytes"]), pinned(batch["out_bytes"]), pinned(16 * n)
            h_in[:] = d_in.cpu().numpy()
            eng.seal_batch(recs, h_in, np.zeros(16, np.uint8), h_out, h_tags)
            t0 = time.perf_counter()
            for _ in range(3):
                eng.seal_batch(recs, h_in, np.zeros(16, np.uint8), h_out, h_tags)
            result["pcie_inclusive_GiBps"] = round(3 * payload / (time.perf_counter() - t0) / 2**30, 3)
            # the same pinned buffers read and written in place by the kernels (ATLS_ZERO_COPY=1), or
            # inputs staged in chunks and outputs written in place (=2)
            for mode, key in ((1, "pcie_zero_copy"), (2, "pcie_zero_copy_out")):
                os.environ["ATLS_ZERO_COPY"] = str(mode)
                zeng = atls.Engine(local)
                del os.environ["ATLS_ZERO_COPY"]
                zeng.set_keys(batch["keys"])
                z_out, z_tags = pinned(batch["out_bytes"]), pinned(16 * n)
                zeng.seal_batch(recs, h_in, np.zeros(16, np.uint8), z_out, z_tags)
                t0 = time.perf_counter()
                for _ in range(3):
                    zeng.seal_batch(recs, h_in, np.zeros(16, np.uint8), z_out, z_tags)
                result[key + "_GiBps"] = round(3 * payload / (time.perf_counter() - t0) / 2**30, 3)
                result[key + "_equal"] = bool(np.array_equal(z_out, h_out) and np.array_equal(z_tags, h_tags))
                zeng.close()
    if args.wire and world == 1 and rank == 0:
        # record framing on the device: header || ct || tag back to back
        wb = workload.wire_batch(batch)
        d_wout = torch.empty(wb["out_bytes"] + 16, dtype=torch.uint8, device=dev)
        d_wrecs = torch.from_numpy(wb["recs"].view(np.uint8).copy()).to(dev)
        w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i in range(args.warmup + args.steps):
            if i == args.warmup:
                eng.join()
                w0.record(stream)
            eng.seal_batch(d_wrecs.data_ptr(), d_in, d_aux, d_wout, None, flags=flags, n=n)
        eng.join()
        w1.record(stream)
        sync()
        result["wire_GiBps"] = round(payload * args.steps / (w0.elapsed_time(w1) * 1e-3) / 2**30, 3)
    del m, d_in, d_out, d_tags
    torch.cuda.empty_cache()
    if world > 1 and not args.no_scatter:
        # A batch arriving at one GPU: the config's WHOLE batch (C4: 1 Mi records, 17 GB
        # each way) on rank 0, split by cumulative bytes over all ranks, scattered over RCCL, sealed by
        # every rank's engine and gathered back (dist.seal_sharded); reported beside `value`, which is
        # the pre-sharded rate. The result must equal rank 0's own single-GPU seal of the whole batch.
        # A failed exchange is recorded in the line; a hung one fires the watchdog on every rank,
        # rank 0 first printing the line without it, and the process exits non-zero
        # (dist.WATCHDOG_EXIT): the measured line survives, and the status says something hung.
        def give_up():
            if rank == 0 and result is not None:
                result["sharded_from_rank0"] = {"error": f"no result within {args.scatter_timeout:.0f} s"}
                print(json.dumps(result), flush=True)

        def exchange():
            whole = whole_batch(args, world)
            eng.set_keys(whole["keys"])
            g = torch.Generator(device=dev).manual_seed(workload.SEEDS["payload"])

            def seal(rr, inp, o, t):
                eng.seal_batch(rr, inp, d_aux, o, t, flags=atls.FLAG_DEVICE_PTRS)  # synchronous

            return sharded_exchange(
                whole, seal, lambda nb: torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=g),
                lambda nb: torch.zeros(nb, dtype=torch.uint8, device=dev), lambda: torch.cuda.synchronize(dev), dev)

        ok, sg = dist.run_or_exit(exchange, args.scatter_timeout, give_up)
        if not ok:
            print(f"sharded exchange failed: {sg}", file=sys.stderr, flush=True)
            sg = {"error": str(sg)[:200]}  # recorded in the line; the measured value stands
        if rank == 0 and result is not None:
            result["sharded_from_rank0"] = sg
        torch.cuda.empty_cache()
    if not args.no_configs:
        # the other BASELINE configs, each rank its own shard, fewer steps
        steps, warmup = min(args.steps, args.config_steps), min(args.warmup, 2)
        cfgs = {}
        for name in EXTRA_CONFIGS:
            if name == args.config:
                continue
            mm = measure(name, eng, dev, rank, world, steps, warmup, not args.no_lazy_join, settle_ms=args.settle_ms,
                         load_settle_ms=args.load_settle_ms)
            cfgs[name] = config_summary(name, mm, steps)
            del mm
        if not args.key_slots:
            # SURVEY §8(d)'s worst case: C2 with a key per record (65,536 connections), so no lane groups form
            name = "c2_aes128gcm_64Ki_x_16KiB"
            mm = measure(name, eng, dev, rank, world, steps, warmup, not args.no_lazy_join,
                         key_slots=workload.CONFIGS[name][1], settle_ms=args.settle_ms,
                         load_settle_ms=args.load_settle_ms)
            cfgs[name + " (a key per record)"] = config_summary(name, mm, steps)
            del mm
        if world == 1 and not args.records:
            # C4 at its stated size on one GPU: the whole 1 Mi x 16 KiB batch (17.2 GB in, 17.2 GB out) in one
            # device-resident launch -- what the 8-GPU config's root holds before it scatters
            name = "c4_aes256gcm_1Mi_x_16KiB"
            mm = measure(name, eng, dev, rank, world, min(steps, 5), min(warmup, 1), not args.no_lazy_join,
                         records=workload.CONFIGS[name][1], settle_ms=args.settle_ms,
                         load_settle_ms=args.load_settle_ms)
            cfgs[name + " (whole batch, 1 GPU)"] = config_summary(name, mm, min(steps, 5))
            del mm
            torch.cuda.empty_cache()
            # C5 likewise: the whole 256 Ki-record mixed batch (2.16 GB each way) in one planned launch
            name = "c5_mixed_256Ki_x_64B-16KiB"
            mm = measure(name, eng, dev, rank, world, steps, warmup, not args.no_lazy_join,
                         records=workload.CONFIGS[name][1], settle_ms=args.settle_ms,
                         load_settle_ms=args.load_settle_ms)
            cfgs[name + " (whole batch, 1 GPU)"] = config_summary(name, mm, steps)
            del mm
            torch.cuda.empty_cache()
        if rank == 0:
            result["configs"] = cfgs
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    dist.close()
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
