// How the batched socket path (stream.cpp) cuts its work into engine batches -- host-only, no HIP, so the
// sanitizer tests (tests/native/batches_fuzz.cpp) check the same code:
//   * a receive round opens whole connections, at most kBatchBytes of wire bytes per batch (one connection more
//     than that is a batch of its own);
//   * a flush seals runs of consecutive records, a quarter of the flush each but 8 .. 64 MiB (smaller flushes are
//     one batch), so one batch is sealed while the previous one is sent;
//   * the connections whose wire bytes a flush batch holds are the ones a sender sends from it.
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace atls_stream {

constexpr size_t kBatchBytes = size_t(64) << 20;
constexpr size_t kMinBatchBytes = size_t(8) << 20;  // a flush's smallest engine batch (if it has that much)

// [c0, c1) ranges of connections whose wire bytes (prefix sums `base`, nc + 1 entries) fit `cap`, skipping empty ones
inline std::vector<std::pair<size_t, size_t>> connection_batches(const std::vector<size_t>& base,
                                                                 size_t cap = kBatchBytes) {
  std::vector<std::pair<size_t, size_t>> g;
  const size_t nc = base.size() - 1;
  for (size_t c0 = 0; c0 < nc;) {
    while (c0 < nc && base[c0 + 1] == base[c0]) c0++;
    if (c0 == nc) break;
    size_t c1 = c0 + 1;
    while (c1 < nc && base[c1 + 1] - base[c0] <= cap) c1++;
    g.emplace_back(c0, c1);
    c0 = c1;
  }
  return g;
}

// The batch size a flush of `total` wire bytes aims at.
inline size_t flush_target(size_t total, size_t cap = kBatchBytes, size_t floor = kMinBatchBytes) {
  return std::min(cap, std::max(floor, total / 4));
}

// First record of each flush batch, then n: records [gs[k], gs[k+1]) hold at most `target` wire bytes (one larger
// record is a batch of its own). wire(r) = record r's wire bytes.
template <class Wire>
inline std::vector<size_t> record_batches(size_t n, size_t target, Wire wire) {
  std::vector<size_t> gs{0};
  for (size_t r = 0, acc = 0; r < n; r++) {
    const size_t w = wire(r);
    if (acc && acc + w > target) {
      gs.push_back(r);
      acc = 0;
    }
    acc += w;
  }
  gs.push_back(n);
  return gs;
}

// [c_lo, c_hi): the connections with wire bytes in [w0, w1) (w0 < w1 <= base.back(); base as above). Empty
// connections inside the range are included (they have nothing to send).
inline std::pair<size_t, size_t> connections_in(const std::vector<size_t>& base, size_t w0, size_t w1) {
  const size_t nc = base.size() - 1;
  const size_t c_lo = (size_t)(std::upper_bound(base.begin(), base.end(), w0) - base.begin()) - 1;
  size_t c_hi = c_lo;
  while (c_hi < nc && base[c_hi] < w1) c_hi++;
  return {c_lo, c_hi};
}

}  // namespace atls_stream
