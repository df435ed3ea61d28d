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
#include <hip/hip_runtime.h>
#include <sys/socket.h>
#include <sys/types.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/atls.h"
#include "record_split.h"

namespace {

constexpr size_t kMaxFragment = size_t(1) << 14;  // RFC 8446 §5.1
constexpr int kUnexpectedMessage = 10;            // TlsError::UnexpectedMessage, alert.rs:22
constexpr int kBrokenPipe = 254;                  // TlsError::BrokenPipe, alert.rs:44


// Grow-only page-locked host buffer: the engine's copies from it run at full PCIe speed.
struct Pinned {
  uint8_t* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t n) {
    if (n <= cap) return true;
    size_t c = cap ? cap : (size_t(1) << 20);
    while (c < n) c *= 2;
    void* q = nullptr;
    if (hipHostMalloc(&q, c, hipHostMallocDefault) != hipSuccess) return false;
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

struct Conn {
  int fd = -1;
  uint32_t wslot = 0, rslot = 0;  // key slots: write key, read key
  uint64_t wseq = 0, rseq = 0;
  int err = 0;                    // TlsError that ended the connection
  std::vector<Record> out;        // queued for the next flush
  std::vector<uint8_t> rx;        // received bytes not yet split into records
  std::vector<uint8_t> wire;      // whole received records waiting for open_pending
  std::vector<uint32_t> offs;     // their offsets in wire
  std::deque<Record> inbox;       // opened records
};

bool send_all(int fd, const uint8_t* p, size_t n) {
  while (n) {
    const ssize_t k = send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= (size_t)k;
  }
  return true;
}

// Moves the whole records at the front of c.rx to c.wire (record_split.h, Record::from_raw checks).
void split(Conn& c) {
  const size_t pos = atls_split::split_records(c.rx.data(), c.rx.size(), c.wire, c.offs, c.err);
  c.rx.erase(c.rx.begin(), c.rx.begin() + (std::ptrdiff_t)pos);
}

}  // namespace

struct atls_stream_batch {
  atls_engine* e = nullptr;
  std::vector<atls_key> keys;  // 2 slots per connection
  bool keys_dirty = false;
  std::vector<Conn> conns;
  Pinned in, wire, pt;
  std::vector<atls_rec> recs;
  std::vector<atls_open_result> res;
  std::mutex mu;
};

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

}  // namespace

extern "C" {

atls_stream_batch* atls_sb_create(atls_engine* e) {
  if (!e) return nullptr;
  atls_stream_batch* sb = new (std::nothrow) atls_stream_batch();
  if (sb) sb->e = e;
  return sb;
}

void atls_sb_destroy(atls_stream_batch* sb) { delete sb; }

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
  sb->conns.push_back(std::move(c));
  return (int)sb->conns.size() - 1;
}

int atls_sb_write(atls_stream_batch* sb, int conn, uint8_t content_type, const uint8_t* data, size_t len) {
  if (!sb || (len && !data) || content_type == 0 || !atls_split::record_type_ok(content_type))
    return ATLS_ILLEGAL_PARAMETER;
  std::lock_guard<std::mutex> lk(sb->mu);
  if (!valid_conn_locked(sb, conn)) return ATLS_ILLEGAL_PARAMETER;
  Conn& c = sb->conns[(size_t)conn];
  if (c.err) return c.err;
  if (len == 0) c.out.push_back(Record{content_type, {}});
  for (size_t off = 0; off < len; off += kMaxFragment) {
    const size_t k = std::min(kMaxFragment, len - off);
    c.out.push_back(Record{content_type, std::vector<uint8_t>(data + off, data + off + k)});
  }
  return ATLS_OK;
}

long atls_sb_flush(atls_stream_batch* sb) {
  if (!sb) return -ATLS_INTERNAL_ERROR;
  std::lock_guard<std::mutex> lk(sb->mu);
  size_t n = 0, in_bytes = 0, wire_bytes = 0;
  for (const Conn& c : sb->conns)
    for (const Record& r : c.out) {
      n++;
      in_bytes += r.data.size();
      wire_bytes += r.data.size() + 22;  // header 5, inner type 1, tag 16
    }
  if (n == 0) return 0;
  if (n > 0xffffffffu) return -ATLS_ILLEGAL_PARAMETER;
  int rc = install_keys(sb);
  if (rc) return -rc;
  if (!sb->in.reserve(in_bytes + 16) || !sb->wire.reserve(wire_bytes + 16)) return -ATLS_INTERNAL_ERROR;
  sb->recs.assign(n, atls_rec{});
  size_t i = 0, io = 0, wo = 0;
  for (Conn& c : sb->conns) {
    uint64_t seq = c.wseq;
    for (const Record& r : c.out) {
      if (!r.data.empty()) std::memcpy(sb->in.p + io, r.data.data(), r.data.size());
      atls_rec& d = sb->recs[i++];
      d.in_off = io;
      d.out_off = wo;
      d.seq = seq++;
      d.len = (uint32_t)r.data.size();
      d.key_slot = c.wslot;
      d.content_type = r.type;
      d.mode = ATLS_MODE_WIRE;
      io += r.data.size();
      wo += r.data.size() + 22;
    }
  }
  rc = atls_seal_batch(sb->e, sb->recs.data(), (uint32_t)n, sb->in.p, nullptr, sb->wire.p, nullptr, 0);
  if (rc) return -rc;
  wo = 0;
  for (Conn& c : sb->conns) {
    if (c.out.empty()) continue;
    size_t bytes = 0;
    for (const Record& r : c.out) bytes += r.data.size() + 22;
    c.wseq += c.out.size();
    c.out.clear();
    if (!c.err && !send_all(c.fd, sb->wire.p + wo, bytes)) c.err = kBrokenPipe;
    wo += bytes;
  }
  return (long)n;
}

int atls_sb_feed(atls_stream_batch* sb, int conn, const uint8_t* data, size_t len) {
  if (!sb || (len && !data)) return ATLS_ILLEGAL_PARAMETER;
  std::lock_guard<std::mutex> lk(sb->mu);
  if (!valid_conn_locked(sb, conn)) return ATLS_ILLEGAL_PARAMETER;
  Conn& c = sb->conns[(size_t)conn];
  c.rx.insert(c.rx.end(), data, data + len);
  if (!c.err) split(c);
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
  if (k == 0) return 0;
  const int rc = atls_sb_feed(sb, conn, buf.data(), (size_t)k);
  return rc ? -rc : (long)k;
}

long atls_sb_open_pending(atls_stream_batch* sb) {
  if (!sb) return -ATLS_INTERNAL_ERROR;
  std::lock_guard<std::mutex> lk(sb->mu);
  size_t n = 0, wire_bytes = 0, pt_bytes = 0;
  for (const Conn& c : sb->conns) {
    if (c.err || c.offs.empty()) continue;
    n += c.offs.size();
    wire_bytes += c.wire.size();
    pt_bytes += c.wire.size();  // >= the ciphertext bytes
  }
  if (n == 0) return 0;
  int rc = install_keys(sb);
  if (rc) return -rc;
  if (!sb->wire.reserve(wire_bytes + 16) || !sb->pt.reserve(pt_bytes + 16)) return -ATLS_INTERNAL_ERROR;
  sb->recs.assign(n, atls_rec{});
  sb->res.assign(n, atls_open_result{});
  size_t i = 0, wo = 0, po = 0;
  for (Conn& c : sb->conns) {
    if (c.err || c.offs.empty()) continue;
    std::memcpy(sb->wire.p + wo, c.wire.data(), c.wire.size());
    for (size_t j = 0; j < c.offs.size(); j++) {
      const uint8_t* h = c.wire.data() + c.offs[j];
      const uint32_t ct = (((uint32_t)h[3] << 8) | h[4]) - 16;
      atls_rec& d = sb->recs[i++];
      d.in_off = wo + c.offs[j];
      d.out_off = po;
      d.seq = c.rseq + j;
      d.len = ct;
      d.key_slot = c.rslot;
      d.mode = ATLS_MODE_WIRE;
      po += ct;
    }
    wo += c.wire.size();
  }
  rc = atls_open_batch(sb->e, sb->recs.data(), (uint32_t)n, sb->wire.p, nullptr, nullptr, sb->pt.p, sb->res.data(), 0);
  if (rc) return -rc;
  i = 0;
  for (Conn& c : sb->conns) {
    if (c.err || c.offs.empty()) continue;
    for (size_t j = 0; j < c.offs.size(); j++, i++) {
      if (c.err) continue;  // a failed record ends the connection
      const atls_open_result& r = sb->res[i];
      if (r.status) {
        c.err = r.status;
        continue;
      }
      const uint8_t* p = sb->pt.p + sb->recs[i].out_off;
      c.inbox.push_back(Record{r.content_type, std::vector<uint8_t>(p, p + r.content_len)});
    }
    c.rseq += c.offs.size();
    c.wire.clear();
    c.offs.clear();
  }
  return (long)n;
}

int atls_sb_read(atls_stream_batch* sb, int conn, uint8_t* buf, size_t cap, size_t* out_len) {
  if (!sb || !out_len || (cap && !buf)) return ATLS_ILLEGAL_PARAMETER;
  for (;;) {
    bool pending;
    {
      std::lock_guard<std::mutex> lk(sb->mu);
      if (!valid_conn_locked(sb, conn)) return ATLS_ILLEGAL_PARAMETER;
      Conn& c = sb->conns[(size_t)conn];
      if (!c.inbox.empty()) {
        Record& r = c.inbox.front();
        if (r.type != 23) {  // stream.rs:112-116
          c.inbox.pop_front();
          return kUnexpectedMessage;
        }
        if (r.data.size() > cap) return ATLS_ILLEGAL_PARAMETER;  // kept for a larger buffer
        if (!r.data.empty()) std::memcpy(buf, r.data.data(), r.data.size());
        *out_len = r.data.size();
        c.inbox.pop_front();
        return ATLS_OK;
      }
      if (c.err) return c.err;
      pending = !c.offs.empty();
    }
    if (pending) {
      const long k = atls_sb_open_pending(sb);
      if (k < 0) return (int)-k;
    } else {
      const long k = atls_sb_recv(sb, conn, size_t(1) << 20);
      if (k == 0) return kBrokenPipe;
      if (k < 0) return (int)-k;
      // take whatever else has arrived before opening, so one batch covers it all
      int fd;
      {
        std::lock_guard<std::mutex> lk(sb->mu);
        fd = sb->conns[(size_t)conn].fd;
      }
      thread_local std::vector<uint8_t> more(size_t(1) << 20);
      for (;;) {
        const ssize_t m = recv(fd, more.data(), more.size(), MSG_DONTWAIT);
        if (m <= 0) break;  // EAGAIN, EOF (seen by the next blocking read) or an error
        const int rc = atls_sb_feed(sb, conn, more.data(), (size_t)m);
        if (rc) return rc;
      }
    }
  }
}

}  // extern "C"
