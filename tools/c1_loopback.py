"""BASELINE.json config C1: server_https-style loopback. A 1 MiB response body goes out as 64
TLS 1.3 records of 16 KiB (TLS_AES_128_GCM_SHA256) over a TCP socket on 127.0.0.1: the server
thread seals and writes, the client reads, splits the stream into records and opens them.
Keys: RFC 8448 §3 server handshake traffic secret -> write key / iv (Key::from_hkdf,
net/key_schedule.rs:40-50), sequence numbers 0..63.

The GPU path of the loop, checked end to end (body and content types); the reference's
per-record CPU path over the same loop is bench.py's cpu_baseline for this config
(`python bench.py --config c1_server_https_loopback_1MiB`):
  * gpu  — atls_derive_keys, then anothertls_amd.stream.StreamBatch on each side: the writes of
           a body (of every connection, with --conns N) sealed in one WIRE-mode atls_seal_batch
           (the device writes header || ct || tag), the received records opened in one
           atls_open_batch (net/stream.rs:97-150 batched);
Prints one JSON line: MB/s of body through seal -> socket -> open.
python tools/c1_loopback.py [--reps N] [--conns N]"""
import argparse
import json
import os
import socket
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

SECRET = bytes.fromhex("b67b7d690cc16c4e75e54213cb2d37b4e9c912bcded9105d42befd59d391ad38")  # RFC 8448 §3
N_REC, CONTENT = 64, 16384


def _pair():
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    cli = socket.create_connection(srv.getsockname())
    conn, _ = srv.accept()
    srv.close()
    for s in (cli, conn):
        s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
    return conn, cli


def _recv_exact(sock, n):
    buf = bytearray(n)
    view, got = memoryview(buf), 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if not k:
            raise ConnectionError("peer closed")
        got += k
    return bytes(buf)


def _loop(seal_body, open_wire, wire_len, reps):
    """reps x (server: seal + send | client: recv + open); returns (seconds, last plaintext)."""
    server, client = _pair()
    out = {}

    def serve():
        for _ in range(reps):
            server.sendall(seal_body())

    t0 = time.perf_counter()
    th = threading.Thread(target=serve)
    th.start()
    for _ in range(reps):
        out["pt"] = open_wire(_recv_exact(client, wire_len))
    th.join()
    dt = time.perf_counter() - t0
    server.close()
    client.close()
    return dt, out["pt"]


def _tcp_pairs(n):
    return [_pair() for _ in range(n)]


def run_gpu(body, reps, conns=1):
    """conns connections over 127.0.0.1, each sending `body` per rep through one StreamBatch per
    side (anothertls_amd/stream.py): the server's writes of all connections are sealed in one
    WIRE-mode batch, the client opens all connections' records in one batch."""
    import anothertls_amd as atls
    from anothertls_amd import stream

    eng_s, eng_c = atls.Engine(0), atls.Engine(0)
    key = eng_s.derive_keys(0x1301, SECRET)[0]  # RFC 8448 server write key (Key::from_hkdf)
    wkey = (0x1301, bytes(key["key"][:16]), bytes(key["static_iv"]))
    pairs = _tcp_pairs(conns)
    srv, cli = stream.StreamBatch(eng_s), stream.StreamBatch(eng_c)
    sc = [srv.add_connection(a, wkey, wkey) for a, _ in pairs]
    cc = [cli.add_connection(b, wkey, wkey) for _, b in pairs]
    wire_len = N_REC * (5 + CONTENT + 1 + 16)
    frags = [body[i * CONTENT:(i + 1) * CONTENT] for i in range(N_REC)]

    def serve(n):
        for _ in range(n):
            for c in sc:
                for f in frags:  # one tls_write per 16 KiB record, as server_https writes
                    srv.tls_write(c, f)
            srv.flush()

    def client(n):
        got = None
        for _ in range(n):
            for c in cc:  # receive every connection's records, then open them all in one batch
                have = 0
                while have < wire_len:
                    data = c.sock.recv(min(1 << 20, wire_len - have))
                    if not data:
                        raise ConnectionError("peer closed")
                    cli.feed(c, data)
                    have += len(data)
            cli.open_pending()
            for c in cc:
                got = b"".join(cli.tls_read(c) for _ in range(N_REC))
        return got

    def run(n):
        th = threading.Thread(target=serve, args=(n,))
        t0 = time.perf_counter()
        th.start()
        pt = client(n)
        th.join()
        return time.perf_counter() - t0, pt

    run(1)  # warm-up (device buffers, code objects, pinned staging)
    dt, pt = run(reps)
    for a, b in pairs:
        a.close()
        b.close()
    eng_s.close()
    eng_c.close()
    return dt, pt


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=8)
    p.add_argument("--conns", type=int, default=1, help="connections sharing one batch")
    args = p.parse_args()
    body = np.random.default_rng(0xC1).integers(0, 256, N_REC * CONTENT, dtype=np.uint8).tobytes()
    dt, pt = run_gpu(body, args.reps, args.conns)
    assert pt == body
    print(json.dumps({"config": "c1_server_https_loopback_1MiB", "records": N_REC, "suite": "TLS_AES_128_GCM_SHA256",
                      "body_bytes": len(body), "gpu_conns": args.conns,
                      "gpu_MBps": round(args.reps * args.conns * len(body) / dt / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
