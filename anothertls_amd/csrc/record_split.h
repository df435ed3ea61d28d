// Splitting a received byte stream into whole TLS records (Record::from_raw, net/record.rs:81-102),
// host-only and HIP-free so that it also builds under ASan / UBSan on the CPU
// (tests/native/split_fuzz.cpp). Used by the batched socket path (stream.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace atls_split {

constexpr int kDecodeError = 51;  // TlsError::DecodeError, net/alert.rs

inline bool record_type_ok(uint32_t b) { return b == 0 || (b >= 20 && b <= 23); }  // RecordType::new, record.rs:23-32

// The whole records at the front of rx[0, n): appends each record's offset (its position in rx plus
// `base`) to offs and returns the bytes they span; the bytes stay where they are (the batched socket
// path opens them in place). A partial record at the end waits for more bytes (the reference has a
// todo!() there, stream.rs:106-108). A complete header whose type is not a RecordType, or that frames
// fewer bytes than a tag (the reference's fragment[..len-16] would underflow, record.rs:208), stops the
// scan with err = DecodeError. The reference's bounds check is 2 + len (record.rs:88); this takes only
// whole 5 + len byte records.
inline size_t scan_records(const uint8_t* rx, size_t n, size_t base, std::vector<uint32_t>& offs, int& err) {
  size_t pos = 0;
  while (n - pos >= 5) {
    const uint8_t* h = rx + pos;
    const size_t len = ((size_t)h[3] << 8) | h[4];
    if (n - pos < 5 + len) break;  // partial record
    if (!record_type_ok(h[0]) || len < 16) {
      err = kDecodeError;
      break;
    }
    offs.push_back((uint32_t)(base + pos));
    pos += 5 + len;
  }
  return pos;
}

// As scan_records, with the whole records moved (appended) to wire and their offsets in wire.
inline size_t split_records(const uint8_t* rx, size_t n, std::vector<uint8_t>& wire, std::vector<uint32_t>& offs,
                            int& err) {
  const size_t used = scan_records(rx, n, wire.size(), offs, err);
  wire.insert(wire.end(), rx, rx + used);
  return used;
}

}  // namespace atls_split
