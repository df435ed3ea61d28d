// Batched TLS 1.3 record streams over sockets, native: TlsStream::tls_write / tls_read
// (net/stream.rs:32-150) for many connections per engine batch.
//
// Every connection queues its records; atls_sb_flush seals the queued records of ALL
// connections in one ATLS_MODE_WIRE batch -- the record kernels write header || ciphertext ||
// tag (RecordPayloadProtection::encrypt, record.rs:162-198) into one page-locked buffer -- and
// sends each connection's slice. Received bytes are split into whole records (Record::from_raw,
// record.rs:81-102; a partial record waits for more bytes where the reference has a todo!() at
// stream.rs:106-108) and atls_sb_open_pending opens the complete records of all connections in
// one batch (the received header is the AAD, record.rs:219; the tag is read from the record).
// Per connection: a write key and a read key, each with its own sequence number
// (Key::get_per_record_nonce, key_schedule.rs:51-64). A record that fails to open ends its
// connection with the reference's error (DecryptError / DecodeError, record.rs:222, :232);
// atls_sb_read returns application data only (UnexpectedMessage otherwise, stream.rs:112-116).
// Divergence (documented): writes longer than 2^14 bytes are fragmented into 2^14-byte records
// (RFC 8446 §5.1); the reference emits one over-long record. Writes up to 2^14 bytes produce the
// reference's wire bytes.
//
// Throughput (round 5): the host work around the device batch is copies and socket
// calls, so the batch keeps them few and spreads them over worker threads (atls_sb_set_threads):
//   * a write is copied once, into the batch's page-locked input arena the seal batch reads; a flush takes
//     that arena and seals and sends from it outside the batch lock, so writes for the next flush (another
//     thread's) fill the second arena meanwhile;
//   * flush sends the connections' slices of the page-locked wire buffer from T threads;
//   * atls_sb_recv_all receives on every connection from T threads, straight into each connection's
//     receive buffer, where the whole records are found in place (record_split.h scan_records);
//   * atls_sb_open_pending gathers the connections' whole records into the page-locked wire buffer,
//     opens them in one batch and hands each connection its plaintexts, both from T threads;
//   * a connection's opened records sit behind its own lock, so readers of different connections
//     (atls_sb_read / atls_sb_read_ready) copy out in parallel.
#include <hip/hip_runtime.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/types.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cerrno>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/atls.h"
#include "record_split.h"
#include "stream_batches.h"

namespace {

constexpr size_t kMaxFragment = size_t(1) << 14;  // RFC 8446 §5.1
constexpr int kUnexpectedMessage = 10;            // TlsError::UnexpectedMessage, alert.rs:22
constexpr int kBrokenPipe = 254;                  // TlsError::BrokenPipe, alert.rs:44
constexpr size_t kRecvChunk = size_t(256) << 10;  // room made in a receive buffer per recv call
constexpr size_t kRxMax = size_t(1) << 31;        // unopened bytes per connection (record offsets are u32)
constexpr int kMaxThreads = 64;

// Grow-only page-locked host buffer: the engine's copies from it run at full PCIe speed. keep: bytes
// [0, keep) survive a growth (the write arena fills across several writes).
struct Pinned {
  uint8_t* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t n, size_t keep = 0) {
    if (n <= cap) return true;
    size_t c = cap ? cap : (size_t(1) << 20);
    while (c < n) c *= 2;
    void* q = nullptr;
    if (hipHostMalloc(&q, c, hipHostMallocDefault) != hipSuccess) return false;
    if (p && keep) std::memcpy(q, p, keep);
    if (p) (void)hipHostFree(p);
    p = (uint8_t*)q;
    cap = c;
    return true;
  }
  ~Pinned() {
    if (p) (void)hipHostFree(p);
  }
};

struct Record {
  uint8_t type;
  std::vector<uint8_t> data;
};

struct Queued {  // a record waiting for the next flush; its content is in the batch's input arena
  size_t in_off;
  uint32_t len;
  uint8_t type;
};

struct Inbox {  // opened records of one connection (its own lock: readers of different connections run in parallel)
  std::mutex mu;
  std::deque<Record> q;
  int err = 0;  // the connection's error, visible to readers once every record before it was handed over
};

struct Conn {
  int fd = -1;
  uint32_t wslot = 0, rslot = 0;  // key slots: write key, read key
  uint64_t wseq = 0, rseq = 0;
  int err = 0;                    // TlsError that ended the connection (batch side)
  bool eof = false;               // the peer closed (recv returned 0)
  std::vector<Queued> out;        // queued for the next flush
  std::vector<uint8_t> rx;        // received bytes [0, rx_len); whole records at offs, scanned up to rx_done
  size_t rx_len = 0, rx_done = 0;
  std::vector<uint32_t> offs;
  std::unique_ptr<Inbox> inbox{new Inbox};
};

bool send_all(int fd, const uint8_t* p, size_t n) {
  while (n) {
    const ssize_t k = send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {  // a non-blocking socket: wait until it drains
        pollfd q{fd, POLLOUT, 0};
        (void)poll(&q, 1, 1000);
        continue;
      }
      return false;
    }
    p += k;
    n -= (size_t)k;
  }
  return true;
}

// Finds the whole records among the received bytes not yet scanned (record_split.h).
void scan(Conn& c) {
  if (c.err) return;
  c.rx_done += atls_split::scan_records(c.rx.data() + c.rx_done, c.rx_len - c.rx_done, c.rx_done, c.offs, c.err);
}

void append_rx(Conn& c, const uint8_t* data, size_t len) {
  if (c.rx.size() < c.rx_len + len) c.rx.resize(std::max(c.rx_len + len, 2 * c.rx.size()));
  std::memcpy(c.rx.data() + c.rx_len, data, len);
  c.rx_len += len;
}

// Receives what the socket holds (non-blocking) straight into c.rx; returns the bytes received.
size_t drain_socket(Conn& c) {
  size_t got = 0;
  while (!c.err && !c.eof) {
    if (c.rx_len >= kRxMax) break;  // the owner must open before more is read
    if (c.rx.size() < c.rx_len + kRecvChunk) c.rx.resize(std::max(c.rx_len + kRecvChunk, 2 * c.rx.size()));
    const ssize_t k = recv(c.fd, c.rx.data() + c.rx_len, c.rx.size() - c.rx_len, MSG_DONTWAIT);
    if (k > 0) {
      c.rx_len += (size_t)k;
      got += (size_t)k;
      continue;
    }
    if (k == 0) c.eof = true;
    else if (errno == EINTR) continue;
    else if (errno != EAGAIN && errno != EWOULDBLOCK) c.err = kBrokenPipe;
    break;
  }
  scan(c);
  return got;
}

// fn(i) for i in [0, n) on up to `threads` threads (the caller's included), item i on thread i % T.
template <typename F>
void parallel(int threads, size_t n, F fn) {
  const size_t T = std::min<size_t>((size_t)std::max(threads, 1), n);
  if (T <= 1) {
    for (size_t i = 0; i < n; i++) fn(i);
    return;
  }
  std::vector<std::thread> ts;
  ts.reserve(T - 1);
  for (size_t t = 1; t < T; t++)
    ts.emplace_back([&, t] {
      for (size_t i = t; i < n; i += T) fn(i);
    });
  for (size_t i = 0; i < n; i += T) fn(i);
  for (auto& th : ts) th.join();
}

}  // namespace

struct atls_stream_batch {
  atls_engine* e = nullptr;
  std::vector<atls_key> keys;  // 2 slots per connection
  bool keys_dirty = false;
  std::vector<Conn> conns;
  // writes go to arena in[cur]; a flush takes that arena (cur flips) and seals and sends from it without the
  // batch lock, so the next flush's writes fill the other arena meanwhile (flush_mu: one flush at a time, so an
  // arena is never written while a flush still reads it)
  Pinned in[2], wire_out[2], wire, pt;
  int cur = 0;
  size_t in_len = 0;  // bytes of queued writes in in[cur]
  std::vector<atls_rec> recs, frecs;  // open / flush descriptors
  std::vector<atls_open_result> res;
  int threads = 1;
  std::mutex mu, flush_mu;
  // the connections' inboxes (owned by their Conn through a unique_ptr, so a pointer stays valid when conns grows),
  // behind a lock of their own: atls_sb_read_ready finds a connection's inbox without the batch lock, which a
  // receive round or an open batch holds for its whole length
  std::vector<Inbox*> inboxes;
  std::mutex inbox_mu;
  Pinned gather;  // a flush batch's inputs in record order, when interleaved writes left them out of order
  size_t gathered_batches = 0;  // flush batches that needed it (atls_debug_sb_gathered)
  // env ATLS_SB_PROFILE=1: seconds per phase, printed to stderr by atls_sb_destroy
  bool profile = std::getenv("ATLS_SB_PROFILE") != nullptr;
  double t_write = 0, t_seal = 0, t_send = 0, t_recv = 0, t_poll = 0, t_gather = 0, t_open = 0, t_hand = 0;
};

namespace {
struct Stopwatch {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  double lap() {
    const auto n = std::chrono::steady_clock::now();
    const double d = std::chrono::duration<double>(n - t).count();
    t = n;
    return d;
  }
};
}  // namespace

namespace {

int install_keys(atls_stream_batch* sb) {
  if (!sb->keys_dirty) return ATLS_OK;
  const int rc = atls_set_keys(sb->e, sb->keys.data(), (uint32_t)sb->keys.size());
  if (rc == ATLS_OK) sb->keys_dirty = false;
  return rc;
}

// Connection ids are checked under sb->mu: atls_sb_add_connection may grow the vector meanwhile.
bool valid_conn_locked(atls_stream_batch* sb, int conn) { return conn >= 0 && (size_t)conn < sb->conns.size(); }

// A connection's keys as the engine would accept them (engine.cpp key_status, plus the 12-byte
// static IV of Key::from_hkdf, key_schedule.rs:44): rejected at add time, so one bad key cannot
// make every later flush of the batch fail.
int key_check(const atls_key& k) {
  if (k.suite == ATLS_TLS_CHACHA20_POLY1305_SHA256) return (k.key_len == 32 && k.iv_len == 12) ? ATLS_OK : ATLS_ILLEGAL_PARAMETER;
  if (k.suite == ATLS_TLS_AES_128_GCM_SHA256 || k.suite == ATLS_TLS_AES_256_GCM_SHA384)
    return ((k.key_len == 16 || k.key_len == 24 || k.key_len == 32) && k.iv_len == 12) ? ATLS_OK : ATLS_ILLEGAL_PARAMETER;
  return ATLS_INSUFFICIENT_SECURITY;
}

// The connection's error becomes visible to its readers (after the records opened before it). A peer that closed
// (recv returned 0) with no whole record left to open ends the stream for its readers with BrokenPipe, as
// TlsStream::tcp_read does at a zero-byte read (net/stream.rs:68-73) -- a partial record left behind never
// completes; writes stay allowed (a half-closed peer may still read).
void publish_err(Conn& c) {
  std::lock_guard<std::mutex> lk(c.inbox->mu);
  if (c.err && !c.inbox->err) c.inbox->err = c.err;
  if (!c.err && c.eof && c.offs.empty() && !c.inbox->err) c.inbox->err = kBrokenPipe;
}

// Opens the whole records of connections [c0, c1) (wire offsets `wbase`, record counts `rbase`, both prefix
// sums from c0) in one engine batch and hands each connection its plaintexts.
long open_group(atls_stream_batch* sb, size_t c0, size_t c1, const std::vector<size_t>& wbase,
                const std::vector<size_t>& rbase) {
  const size_t n = rbase[c1] - rbase[c0], wire_bytes = wbase[c1] - wbase[c0];
  // plaintexts packed back to back (the engine copies a gapless output range back in one piece)
  if (!sb->wire.reserve(wire_bytes + 16) || !sb->pt.reserve(wire_bytes + 16)) return -ATLS_INTERNAL_ERROR;
  std::vector<size_t> pbase(c1 - c0 + 1, 0);
  for (size_t i = c0; i < c1; i++) {
    size_t ptb = 0;
    const Conn& c = sb->conns[i];
    if (rbase[i + 1] != rbase[i])
      for (uint32_t o : c.offs) ptb += (((size_t)c.rx[o + 3] << 8) | c.rx[o + 4]) - 16;
    pbase[i - c0 + 1] = pbase[i - c0] + ptb;
  }
  sb->recs.assign(n, atls_rec{});
  sb->res.assign(n, atls_open_result{});
  Stopwatch sw;
  parallel(sb->threads, c1 - c0, [&](size_t k) {  // gather each connection's whole records, describe them
    const size_t ci = c0 + k;
    Conn& c = sb->conns[ci];
    if (rbase[ci + 1] == rbase[ci]) return;
    const size_t wb = wbase[ci] - wbase[c0], rb = rbase[ci] - rbase[c0];
    std::memcpy(sb->wire.p + wb, c.rx.data(), c.rx_done);
    size_t po = pbase[k];
    for (size_t j = 0; j < c.offs.size(); j++) {
      const uint8_t* h = c.rx.data() + c.offs[j];
      atls_rec& d = sb->recs[rb + j];
      d.in_off = wb + c.offs[j];
      d.out_off = po;
      po += (((uint32_t)h[3] << 8) | h[4]) - 16;
      d.seq = c.rseq + j;
      d.len = (((uint32_t)h[3] << 8) | h[4]) - 16;
      d.key_slot = c.rslot;
      d.mode = ATLS_MODE_WIRE;
    }
  });
  sb->t_gather += sw.lap();
  const int rc = atls_open_batch(sb->e, sb->recs.data(), (uint32_t)n, sb->wire.p, nullptr, nullptr, sb->pt.p,
                                 sb->res.data(), 0);
  if (rc) return -rc;
  sb->t_open += sw.lap();
  parallel(sb->threads, c1 - c0, [&](size_t k) {  // hand each connection its plaintexts, keep its partial tail
    const size_t ci = c0 + k;
    Conn& c = sb->conns[ci];
    if (rbase[ci + 1] == rbase[ci]) return;
    const size_t rb = rbase[ci] - rbase[c0];
    std::vector<Record> got;
    got.reserve(c.offs.size());
    for (size_t j = 0; j < c.offs.size(); j++) {
      const atls_open_result& r = sb->res[rb + j];
      if (r.status) {  // a failed record ends the connection
        c.err = r.status;
        break;
      }
      const uint8_t* p = sb->pt.p + sb->recs[rb + j].out_off;
      got.push_back(Record{r.content_type, std::vector<uint8_t>(p, p + r.content_len)});
    }
    c.rseq += c.offs.size();
    std::memmove(c.rx.data(), c.rx.data() + c.rx_done, c.rx_len - c.rx_done);
    c.rx_len -= c.rx_done;
    c.rx_done = 0;
    c.offs.clear();
    {
      std::lock_guard<std::mutex> lk(c.inbox->mu);
      for (Record& r : got) c.inbox->q.push_back(std::move(r));
      if (c.err && !c.inbox->err) c.inbox->err = c.err;
      if (!c.err && c.eof && !c.inbox->err) c.inbox->err = kBrokenPipe;  // publish_err: the peer closed
    }
  });
  sb->t_hand += sw.lap();
  return (long)n;
}

long open_pending_locked(atls_stream_batch* sb) {
  const size_t nc = sb->conns.size();
  std::vector<size_t> wbase(nc + 1, 0), rbase(nc + 1, 0);
  for (size_t i = 0; i < nc; i++) {
    const Conn& c = sb->conns[i];
    const bool any = !c.err && !c.offs.empty();
    wbase[i + 1] = wbase[i] + (any ? c.rx_done : 0);
    rbase[i + 1] = rbase[i] + (any ? c.offs.size() : 0);
  }
  const size_t n = rbase[nc];
  if (n == 0) return 0;
  if (n > 0xffffffffu) return -ATLS_ILLEGAL_PARAMETER;
  const int rc = install_keys(sb);
  if (rc) return -rc;
  for (const auto& g : atls_stream::connection_batches(wbase)) {  // a connection that has records pending has wire bytes
    const long got = open_group(sb, g.first, g.second, wbase, rbase);
    if (got < 0) return got;
  }
  return (long)n;
}

// One record of the connection's inbox into buf: ATLS_OK, kUnexpectedMessage for a record that is not
// application data (dropped, stream.rs:112-116), ATLS_ILLEGAL_PARAMETER when it does not fit (kept), the
// connection's error once its inbox is empty, or -1 when nothing is there yet.
int pop_inbox(Inbox& in, uint8_t* buf, size_t cap, size_t* out_len) {
  std::lock_guard<std::mutex> lk(in.mu);
  if (in.q.empty()) return in.err ? in.err : -1;
  Record& r = in.q.front();
  if (r.type != 23) {
    in.q.pop_front();
    return kUnexpectedMessage;
  }
  if (r.data.size() > cap) return ATLS_ILLEGAL_PARAMETER;
  if (!r.data.empty()) std::memcpy(buf, r.data.data(), r.data.size());
  *out_len = r.data.size();
  in.q.pop_front();
  return ATLS_OK;
}

Inbox* inbox_of(atls_stream_batch* sb, int conn) {
  std::lock_guard<std::mutex> lk(sb->inbox_mu);
  return conn >= 0 && (size_t)conn < sb->inboxes.size() ? sb->inboxes[(size_t)conn] : nullptr;
}

}  // namespace

extern "C" {

atls_stream_batch* atls_sb_create(atls_engine* e) {
  if (!e) return nullptr;
  atls_stream_batch* sb = new (std::nothrow) atls_stream_batch();
  if (sb) sb->e = e;
  return sb;
}

void atls_sb_destroy(atls_stream_batch* sb) {
  if (sb && sb->profile)
    std::fprintf(stderr,
                 "atls_sb profile (s): write %.4f seal %.4f send %.4f recv %.4f poll %.4f gather %.4f open %.4f hand %.4f\n",
                 sb->t_write, sb->t_seal, sb->t_send, sb->t_recv, sb->t_poll, sb->t_gather, sb->t_open, sb->t_hand);
  delete sb;
}

int atls_sb_set_threads(atls_stream_batch* sb, int threads) {
  if (!sb || threads < 1 || threads > kMaxThreads) return ATLS_ILLEGAL_PARAMETER;
  std::lock_guard<std::mutex> lk(sb->mu);
  sb->threads = threads;
  return ATLS_OK;
}

int atls_sb_add_connection(atls_stream_batch* sb, int fd, const atls_key* write_key, const atls_key* read_key) {
  if (!sb || !write_key || !read_key) return -ATLS_ILLEGAL_PARAMETER;
  if (const int rc = key_check(*write_key)) return -rc;
  if (const int rc = key_check(*read_key)) return -rc;
  std::lock_guard<std::mutex> lk(sb->mu);
  Conn c;
  c.fd = fd;
  c.wslot = (uint32_t)sb->keys.size();
  c.rslot = c.wslot + 1;
  sb->keys.push_back(*write_key);
  sb->keys.push_back(*read_key);
  sb->keys_dirty = true;
  Inbox* inbox = c.inbox.get();
  sb->conns.push_back(std::move(c));
  {
    std::lock_guard<std::mutex> il(sb->inbox_mu);
    sb->inboxes.push_back(inbox);
  }
  return (int)sb->conns.size() - 1;
}

int atls_sb_write(atls_stream_batch* sb, int conn, uint8_t content_type, const uint8_t* data, size_t len) {
  if (!sb || (len && !data) || content_type == 0 || !atls_split::record_type_ok(content_type))
    return ATLS_ILLEGAL_PARAMETER;
  std::lock_guard<std::mutex> lk(sb->mu);
  if (!valid_conn_locked(sb, conn)) return ATLS_ILLEGAL_PARAMETER;
  Conn& c = sb->conns[(size_t)conn];
  if (c.err) return c.err;
  Stopwatch sw;
  struct Add {
    atls_stream_batch* sb;
    Stopwatch& w;
    ~Add() { sb->t_write += w.lap(); }
  } add{sb, sw};
  Pinned& in = sb->in[sb->cur];
  if (!in.reserve(sb->in_len + len + 16, sb->in_len)) return ATLS_INTERNAL_ERROR;
  if (len) std::memcpy(in.p + sb->in_len, data, len);  // the only copy of the write on the host
  if (len == 0) c.out.push_back(Queued{sb->in_len, 0, content_type});
  for (size_t off = 0; off < len; off += kMaxFragment)
    c.out.push_back(Queued{sb->in_len + off, (uint32_t)std::min(kMaxFragment, len - off), content_type});
  sb->in_len += len;
  return ATLS_OK;
}

long atls_sb_flush(atls_stream_batch* sb) {
  if (!sb) return -ATLS_INTERNAL_ERROR;
  std::lock_guard<std::mutex> fl(sb->flush_mu);
  // under the batch lock: take every connection's queued records and the arena they are in
  std::vector<int> fds;
  std::vector<char> dead;
  std::vector<size_t> wbase, rbase;
  size_t n = 0;
  Pinned* arena = nullptr;
  int threads = 1;
  {
    std::lock_guard<std::mutex> lk(sb->mu);
    const size_t nc = sb->conns.size();
    rbase.assign(nc + 1, 0);
    wbase.assign(nc + 1, 0);
    for (size_t i = 0; i < nc; i++) {
      size_t bytes = 0;
      for (const Queued& r : sb->conns[i].out) bytes += r.len + 22;  // header 5, inner type 1, tag 16
      wbase[i + 1] = wbase[i] + bytes;
      rbase[i + 1] = rbase[i] + sb->conns[i].out.size();
    }
    n = rbase[nc];
    if (n == 0) return 0;
    if (n > 0xffffffffu) return -ATLS_ILLEGAL_PARAMETER;
    const int rc = install_keys(sb);
    if (rc) return -rc;
    // the arena later writes will fill, sized like this one so they do not regrow it (before anything is taken,
    // so a failure leaves the queued records where they are)
    if (!sb->in[sb->cur ^ 1].reserve(sb->in[sb->cur].cap)) return -ATLS_INTERNAL_ERROR;
    sb->frecs.assign(n, atls_rec{});
    fds.resize(nc);
    dead.assign(nc, 0);
    for (size_t ci = 0; ci < nc; ci++) {  // each connection's records back to back on its wire slice
      Conn& c = sb->conns[ci];
      fds[ci] = c.fd;
      dead[ci] = c.err != 0;
      size_t wo = wbase[ci];
      for (size_t j = 0; j < c.out.size(); j++) {
        const Queued& r = c.out[j];
        atls_rec& d = sb->frecs[rbase[ci] + j];
        d.in_off = r.in_off;
        d.out_off = wo;  // made relative to its engine batch below
        d.seq = c.wseq + j;
        d.len = r.len;
        d.key_slot = c.wslot;
        d.content_type = r.type;
        d.mode = ATLS_MODE_WIRE;
        wo += r.len + 22;
      }
      c.wseq += c.out.size();
      c.out.clear();
    }
    arena = &sb->in[sb->cur];
    sb->cur ^= 1;  // later writes fill the other arena
    sb->in_len = 0;
    threads = sb->threads;
  }
  // Engine batches of consecutive records (a quarter of the flush each, 8 .. 64 MiB of wire bytes; smaller flushes
  // are one batch: a 1 MiB flush cut into 256 KiB batches took 4x as long, each batch paying its own copies,
  // launch and wait): batch g is sealed into wire_out[g & 1] while batch g - 1 is sent from the other buffer. A
  // connection's bytes go out in order: its part of batch g - 1 is sent before its part of batch g, and a
  // connection whose send failed sends nothing more.
  const size_t nc = fds.size(), total = wbase[nc];
  const std::vector<size_t> gs = atls_stream::record_batches(  // first record of each batch, then n
      n, atls_stream::flush_target(total), [&](size_t r) { return (size_t)sb->frecs[r].len + 22u; });
  std::vector<size_t> gw(gs.size());  // the batches' first wire bytes, then total
  for (size_t g = 0; g + 1 < gs.size(); g++) gw[g] = sb->frecs[gs[g]].out_off;
  gw.back() = total;
  std::vector<char> failed(nc, 0);
  std::thread sender;
  int rc = ATLS_OK;
  size_t gathered = 0;
  size_t g = 0;
  Stopwatch sw;
  for (; g + 1 < gs.size(); g++) {
    const size_t r0 = gs[g], r1 = gs[g + 1], w0 = gw[g], w1 = gw[g + 1];
    Pinned& out = sb->wire_out[g & 1];
    if (!out.reserve(w1 - w0 + 16)) {
      rc = ATLS_INTERNAL_ERROR;
      break;
    }
    for (size_t r = r0; r < r1; r++) sb->frecs[r].out_off -= w0;
    // The records of a batch are in connection order; their inputs are in write order. When writes were
    // interleaved across connections (a server writing round robin) the inputs are out of order, and the engine
    // would stage the whole arena prefix in one copy instead of pipelining its chunks (engine.cpp
    // run_host_pipelined) -- once per batch. Such a batch's inputs are first gathered in record order.
    const uint8_t* src = arena->p;
    bool ascending = true;
    for (size_t r = r0 + 1; r < r1 && ascending; r++)
      ascending = sb->frecs[r].in_off >= sb->frecs[r - 1].in_off + sb->frecs[r - 1].len;
    if (!ascending) {
      std::vector<size_t> at(r1 - r0 + 1, 0);
      for (size_t r = r0; r < r1; r++) at[r - r0 + 1] = at[r - r0] + sb->frecs[r].len;
      if (!sb->gather.reserve(at.back() + 16)) {
        rc = ATLS_INTERNAL_ERROR;
        break;
      }
      parallel(threads, r1 - r0, [&](size_t k) {
        atls_rec& d = sb->frecs[r0 + k];
        if (d.len) std::memcpy(sb->gather.p + at[k], arena->p + d.in_off, d.len);
        d.in_off = at[k];
      });
      src = sb->gather.p;
      gathered++;
    }
    rc = atls_seal_batch(sb->e, sb->frecs.data() + r0, (uint32_t)(r1 - r0), src, nullptr, out.p, nullptr, 0);
    if (rc) break;
    sb->t_seal += sw.lap();
    if (sender.joinable()) sender.join();
    const auto cr = atls_stream::connections_in(wbase, w0, w1);  // the connections with bytes in [w0, w1)
    const size_t c_lo = cr.first, c_hi = cr.second;
    sender = std::thread([&, c_lo, c_hi, w0, w1, wire = out.p] {
      parallel(threads, c_hi - c_lo, [&](size_t k) {
        const size_t ci = c_lo + k;
        const size_t lo = std::max(wbase[ci], w0), hi = std::min(wbase[ci + 1], w1);
        if (dead[ci] || failed[ci] || hi <= lo) return;
        if (!send_all(fds[ci], wire + (lo - w0), hi - lo)) failed[ci] = 1;
      });
    });
  }
  if (sender.joinable()) sender.join();
  sb->t_send += sw.lap();
  {
    std::lock_guard<std::mutex> lk(sb->mu);
    sb->gathered_batches += gathered;
    for (size_t ci = 0; ci < nc; ci++) {
      Conn& c = sb->conns[ci];
      if (failed[ci] && !c.err) c.err = kBrokenPipe;
      // records of batches the engine did not seal are lost: their connections end with the engine's error
      if (rc && g + 1 < gs.size() && wbase[ci + 1] > gw[g] && wbase[ci + 1] != wbase[ci] && !c.err) c.err = rc;
      publish_err(c);
    }
  }
  return rc ? -rc : (long)n;
}

int atls_sb_feed(atls_stream_batch* sb, int conn, const uint8_t* data, size_t len) {
  if (!sb || (len && !data)) return ATLS_ILLEGAL_PARAMETER;
  std::lock_guard<std::mutex> lk(sb->mu);
  if (!valid_conn_locked(sb, conn)) return ATLS_ILLEGAL_PARAMETER;
  Conn& c = sb->conns[(size_t)conn];
  if (c.rx_len + len > kRxMax) return ATLS_ILLEGAL_PARAMETER;
  if (len) append_rx(c, data, len);
  scan(c);
  publish_err(c);
  return c.err;
}

long atls_sb_recv(atls_stream_batch* sb, int conn, size_t max_bytes) {
  if (!sb || max_bytes == 0) return -ATLS_ILLEGAL_PARAMETER;
  int fd;
  {
    std::lock_guard<std::mutex> lk(sb->mu);
    if (!valid_conn_locked(sb, conn)) return -ATLS_ILLEGAL_PARAMETER;
    fd = sb->conns[(size_t)conn].fd;
  }
  thread_local std::vector<uint8_t> buf;  // reused: a fresh vector would zero max_bytes per call
  if (buf.size() < max_bytes) buf.resize(max_bytes);
  ssize_t k;
  do {
    k = recv(fd, buf.data(), max_bytes, 0);
  } while (k < 0 && errno == EINTR);
  if (k < 0) return -kBrokenPipe;
  if (k == 0) {
    std::lock_guard<std::mutex> lk(sb->mu);
    Conn& c = sb->conns[(size_t)conn];
    c.eof = true;
    publish_err(c);
    return 0;
  }
  const int rc = atls_sb_feed(sb, conn, buf.data(), (size_t)k);
  return rc ? -rc : (long)k;
}

long atls_sb_recv_all(atls_stream_batch* sb, int timeout_ms) {
  if (!sb) return -ATLS_INTERNAL_ERROR;
  std::unique_lock<std::mutex> lk(sb->mu);
  Stopwatch sw;
  for (int round = 0; round < 2; round++) {
    const size_t nc = sb->conns.size();
    std::atomic<size_t> total{0};
    parallel(sb->threads, nc, [&](size_t ci) { total += drain_socket(sb->conns[ci]); });
    for (Conn& c : sb->conns) publish_err(c);
    sb->t_recv += sw.lap();
    if (total.load() || timeout_ms <= 0 || round) return (long)total.load();
    std::vector<pollfd> fds;  // nothing arrived: wait for any open connection, once, without the batch lock
    for (const Conn& c : sb->conns)
      if (!c.err && !c.eof && c.rx_len < kRxMax) fds.push_back(pollfd{c.fd, POLLIN, 0});
    if (fds.empty()) return 0;
    lk.unlock();
    const int pr = poll(fds.data(), fds.size(), timeout_ms);
    lk.lock();
    sb->t_poll += sw.lap();
    if (pr <= 0) return 0;
  }
  return 0;
}

long atls_sb_open_pending(atls_stream_batch* sb) {
  if (!sb) return -ATLS_INTERNAL_ERROR;
  std::lock_guard<std::mutex> lk(sb->mu);
  return open_pending_locked(sb);
}

int atls_sb_read_ready(atls_stream_batch* sb, int conn, uint8_t* buf, size_t cap, size_t* out_len) {
  if (!sb || !out_len || (cap && !buf)) return ATLS_ILLEGAL_PARAMETER;
  Inbox* in = inbox_of(sb, conn);
  if (!in) return ATLS_ILLEGAL_PARAMETER;
  // the inbox outlives a conns growth (it is owned through a pointer), so it is read without sb->mu
  const int rc = pop_inbox(*in, buf, cap, out_len);
  return rc < 0 ? ATLS_WOULD_BLOCK : rc;
}

int atls_sb_read(atls_stream_batch* sb, int conn, uint8_t* buf, size_t cap, size_t* out_len) {
  if (!sb || !out_len || (cap && !buf)) return ATLS_ILLEGAL_PARAMETER;
  for (;;) {
    const int rc = atls_sb_read_ready(sb, conn, buf, cap, out_len);
    if (rc != ATLS_WOULD_BLOCK) return rc;
    bool pending, eof;
    {
      std::lock_guard<std::mutex> lk(sb->mu);
      Conn& c = sb->conns[(size_t)conn];
      if (c.err) {
        publish_err(c);
        continue;  // the error reaches the reader after the records before it
      }
      pending = !c.offs.empty();
      eof = c.eof;
    }
    if (pending) {
      const long k = atls_sb_open_pending(sb);
      if (k < 0) return (int)-k;
    } else if (eof) {
      return kBrokenPipe;
    } else {
      const long k = atls_sb_recv(sb, conn, size_t(1) << 20);
      if (k == 0) return kBrokenPipe;
      if (k < 0) return (int)-k;
      // take whatever else has arrived before opening, so one batch covers it all
      std::lock_guard<std::mutex> lk(sb->mu);
      drain_socket(sb->conns[(size_t)conn]);
      publish_err(sb->conns[(size_t)conn]);
    }
  }
}

// Diagnostic: flush batches whose inputs were gathered into record order (interleaved writes; tests).
unsigned long long atls_debug_sb_gathered(atls_stream_batch* sb) {
  if (!sb) return 0;
  std::lock_guard<std::mutex> lk(sb->mu);
  return sb->gathered_batches;
}

}  // extern "C"
