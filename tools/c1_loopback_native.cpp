// BASELINE config C1 (server_https over loopback), native: a server thread sends `reps` bodies of
// 1 MiB (64 records of 16 KiB, TLS_AES_128_GCM_SHA256) on each of `conns` TCP connections over
// 127.0.0.1 through one atls_stream_batch (every body's records of every connection sealed in
// one WIRE-mode batch); the client receives through another batch, which opens every
// connection's pending records together, and checks every byte. Keys: the RFC 8448 §3 server
// handshake traffic secret through atls_derive_keys (Key::from_hkdf, key_schedule.rs:40-50).
// Prints one JSON line: MB/s of body through seal -> socket -> open.
// With threads > 1 (C1 at scale) both batches use that many worker threads
// (atls_sb_set_threads): the server's flush sends from T threads; the client receives every connection
// with atls_sb_recv_all, opens everything pending in one batch, and T reader threads take the opened
// records of their connections (atls_sb_read_ready) and compare every byte; the server writes the next bodies
// on one thread while another flushes the last ones. phase_ms: each side's time per phase over the timed run
// (the two sides overlap, so they do not sum to wall).
//
// Built by __graft_entry__.build() with tools/build_native.sh (g++, linked to libatls.so).
// Usage: tools/c1_loopback_native [reps=8] [conns=1] [threads=1]
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "atls.h"

namespace {

constexpr int kRecords = 64;
constexpr size_t kContent = 16384;
constexpr size_t kBody = kRecords * kContent;

bool tcp_pair(int* server_fd, int* client_fd) {
  const int ls = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  socklen_t al = sizeof a;
  if (ls < 0 || bind(ls, (sockaddr*)&a, sizeof a) || listen(ls, 1) || getsockname(ls, (sockaddr*)&a, &al)) return false;
  const int c = socket(AF_INET, SOCK_STREAM, 0);
  if (c < 0 || connect(c, (sockaddr*)&a, sizeof a)) return false;
  const int s = accept(ls, nullptr, nullptr);
  close(ls);
  if (s < 0) return false;
  const int buf = 4 << 20;
  for (int fd : {s, c}) {
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof buf);
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
  }
  *server_fd = s;
  *client_fd = c;
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 8;
  const int conns = argc > 2 ? std::atoi(argv[2]) : 1;
  const int threads = argc > 3 ? std::atoi(argv[3]) : 1;
  atls_engine* es = atls_engine_create(0);
  atls_engine* ec = atls_engine_create(0);
  if (!es || !ec) {
    std::fprintf(stderr, "c1_loopback_native: no usable HIP device\n");
    return 2;
  }
  static const uint8_t kSecret[32] = {0xb6, 0x7b, 0x7d, 0x69, 0x0c, 0xc1, 0x6c, 0x4e, 0x75, 0xe5, 0x42,
                                      0x13, 0xcb, 0x2d, 0x37, 0xb4, 0xe9, 0xc9, 0x12, 0xbc, 0xde, 0xd9,
                                      0x10, 0x5d, 0x42, 0xbe, 0xfd, 0x59, 0xd3, 0x91, 0xad, 0x38};
  atls_key key;
  if (atls_derive_keys(es, ATLS_TLS_AES_128_GCM_SHA256, kSecret, 32, 1, &key)) return 3;
  std::vector<uint8_t> body(kBody);
  uint64_t x = 0xC1;
  for (auto& b : body) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    b = (uint8_t)x;
  }
  atls_stream_batch* ss = atls_sb_create(es);
  atls_stream_batch* cs = atls_sb_create(ec);
  if (atls_sb_set_threads(ss, threads) || atls_sb_set_threads(cs, threads)) return 5;
  std::vector<int> sc(conns), cc(conns), fds;
  for (int i = 0; i < conns; i++) {
    int s, c;
    if (!tcp_pair(&s, &c)) return 4;
    fds.push_back(s);
    fds.push_back(c);
    sc[i] = atls_sb_add_connection(ss, s, &key, &key);
    cc[i] = atls_sb_add_connection(cs, c, &key, &key);
  }
  std::atomic<bool> ok{true};
  using clk = std::chrono::steady_clock;
  auto secs = [](clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); };
  double t_write = 0, t_flush = 0, t_recv = 0, t_open = 0, t_read = 0;  // phase seconds of the last run
  long flushes = 0, rounds = 0;  // server flushes and client receive rounds of the last run
  auto run = [&](int n) {
    t_write = t_flush = t_recv = t_open = t_read = 0;
    flushes = rounds = 0;
    auto write_rep = [&] {
      const auto t = clk::now();
      for (int i = 0; i < conns; i++)
        for (int k = 0; k < kRecords; k++)  // one tls_write per 16 KiB record
          atls_sb_write(ss, sc[i], 23, body.data() + k * kContent, kContent);
      t_write += secs(t);
    };
    auto flush = [&] {
      const auto t = clk::now();
      if (atls_sb_flush(ss) < 0) ok = false;
      t_flush += secs(t);
    };
    std::thread server([&] {
      if (threads <= 1) {  // write a body on every connection, flush, repeat
        for (int r = 0; r < n; r++) {
          write_rep();
          flush();
          flushes++;
        }
        return;
      }
      // at scale: one thread writes the next bodies while another seals and sends the last ones (a flush
      // takes the queued records and their input arena, so writes go on into the other arena meanwhile)
      // The writer stays at most one body ahead of the flushes (back-pressure, as a server bounds what it
      // queues), so a flush takes one or two bodies and the two input arenas keep their size.
      std::mutex m;
      std::condition_variable cv;
      int written = 0, taken = 0;
      std::thread writer([&] {
        for (int r = 0; r < n; r++) {
          {
            std::unique_lock<std::mutex> lk(m);
            cv.wait(lk, [&] { return taken >= r - 1; });
          }
          write_rep();
          std::lock_guard<std::mutex> lk(m);
          written = r + 1;
          cv.notify_all();
        }
      });
      for (int flushed = 0; flushed < n;) {
        {
          std::unique_lock<std::mutex> lk(m);
          cv.wait(lk, [&] { return written > flushed; });
          flushed = written;
        }
        flush();
        flushes++;
        std::lock_guard<std::mutex> lk(m);
        taken = flushed;
        cv.notify_all();
      }
      writer.join();
      flush();  // anything written after the last counted body (none when reps were counted in order)
    });
    if (threads <= 1) {  // the reference's shape: one tls_read per record, in order
      std::vector<uint8_t> buf(kContent);
      for (int r = 0; r < n; r++)
        for (int i = 0; i < conns; i++)
          for (int k = 0; k < kRecords; k++) {
            size_t got = 0;
            if (atls_sb_read(cs, cc[i], buf.data(), buf.size(), &got) || got != kContent ||
                std::memcmp(buf.data(), body.data() + k * kContent, kContent))
              ok = false;
          }
    } else {  // receive everything pending, open it in one batch, read out on T threads
      std::vector<long> left(conns, (long)n * kRecords);
      long remaining = (long)n * kRecords * conns;
      auto t_idle = std::chrono::steady_clock::now();
      while (remaining > 0 && ok) {
        auto t = clk::now();
        rounds++;
        const long got = atls_sb_recv_all(cs, 100);
        t_recv += secs(t);
        t = clk::now();
        if (got < 0 || atls_sb_open_pending(cs) < 0) {
          ok = false;
          break;
        }
        t_open += secs(t);
        t = clk::now();
        std::atomic<long> taken{0};
        std::vector<std::thread> rd;
        for (int t = 0; t < threads; t++)
          rd.emplace_back([&, t] {
            std::vector<uint8_t> buf(kContent);
            for (int i = t; i < conns; i += threads)
              for (;;) {
                size_t len = 0;
                const int rc = atls_sb_read_ready(cs, cc[i], buf.data(), buf.size(), &len);
                if (rc == ATLS_WOULD_BLOCK) break;
                const long k = (long)n * kRecords - left[i];
                if (rc || len != kContent || std::memcmp(buf.data(), body.data() + (k % kRecords) * kContent, kContent)) {
                  ok = false;
                  return;
                }
                left[i]--;
                taken++;
              }
          });
        for (auto& th : rd) th.join();
        t_read += secs(t);
        remaining -= taken.load();
        if (got > 0 || taken.load() > 0) t_idle = std::chrono::steady_clock::now();
        else if (std::chrono::steady_clock::now() - t_idle > std::chrono::seconds(20)) ok = false;  // stalled
      }
    }
    server.join();
  };
  // warm-up at the timed size: device buffers, code objects and the page-locked arenas grow to what the
  // timed run's batches need (a flush or receive round can take several bodies at once), as in a server that
  // has been running
  run(reps);
  const auto t0 = std::chrono::steady_clock::now();
  run(reps);
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("{\"config\": \"c1_server_https_loopback_1MiB\", \"impl\": \"native atls_stream_batch\", "
              "\"suite\": \"TLS_AES_128_GCM_SHA256\", \"records_per_body\": %d, \"conns\": %d, \"reps\": %d, "
              "\"threads\": %d, \"verified\": %s, \"gpu_MBps\": %.1f, \"phase_ms\": {\"server_write\": %.1f, "
              "\"server_flush\": %.1f, \"client_recv\": %.1f, \"client_open\": %.1f, \"client_read\": %.1f, "
              "\"wall\": %.1f}, \"flushes\": %ld, \"client_rounds\": %ld}\n",
              kRecords, conns, reps, threads, ok.load() ? "true" : "false", (double)reps * conns * kBody / dt / 1e6,
              t_write * 1e3, t_flush * 1e3, t_recv * 1e3, t_open * 1e3, t_read * 1e3, dt * 1e3, flushes, rounds);
  for (int fd : fds) close(fd);
  atls_sb_destroy(ss);
  atls_sb_destroy(cs);
  atls_engine_destroy(es);
  atls_engine_destroy(ec);
  return ok.load() ? 0 : 1;
}
