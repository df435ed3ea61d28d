// TEST INFRASTRUCTURE ONLY. The batched socket path's batch cutting (anothertls_amd/csrc/stream_batches.h, used by
// stream.cpp's flush and receive rounds) on random connection / record layouts, under ASan + UBSan, against the
// invariants the path relies on: every record (connection) in exactly one batch, in order; a batch within its
// size unless it is a single record (connection); a flush batch that stops early only because the next record
// would not fit; the connections a sender sends from a batch are exactly those with bytes in it. Prints OK.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../anothertls_amd/csrc/stream_batches.h"

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAIL line %d: %s\n", __LINE__, #c);    \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

int main() {
  std::mt19937_64 rng(0xBA7C4E5);
  for (int it = 0; it < 20000; it++) {
    const size_t nc = 1 + rng() % 40;
    const size_t cap = 1 + rng() % 5000, floor_ = 1 + rng() % 3000;
    std::vector<size_t> recs_per(nc), wire;  // records of each connection, wire bytes of each record
    std::vector<size_t> base(nc + 1, 0);
    for (size_t c = 0; c < nc; c++) {
      recs_per[c] = (rng() % 4 == 0) ? 0 : rng() % 8;
      size_t b = 0;
      for (size_t j = 0; j < recs_per[c]; j++) {
        const size_t w = 22 + rng() % ((rng() % 8 == 0) ? 9000 : 700);
        wire.push_back(w);
        b += w;
      }
      base[c + 1] = base[c] + b;
    }
    const size_t n = wire.size(), total = base[nc];
    // receive rounds: whole connections
    const auto cg = atls_stream::connection_batches(base, cap);
    size_t next = 0;
    for (const auto& g : cg) {
      CHECK(g.first < g.second && g.second <= nc && g.first >= next);
      for (size_t c = next; c < g.first; c++) CHECK(base[c + 1] == base[c]);  // skipped ones are empty
      CHECK(base[g.first + 1] > base[g.first]);
      CHECK(g.second == g.first + 1 || base[g.second] - base[g.first] <= cap);
      if (g.second < nc) CHECK(base[g.second + 1] - base[g.first] > cap || base[g.second + 1] == base[g.second]);
      next = g.second;
    }
    for (size_t c = next; c < nc; c++) CHECK(base[c + 1] == base[c]);
    // flushes: runs of consecutive records
    const size_t target = atls_stream::flush_target(total, cap, floor_);
    CHECK(target <= cap && (target >= floor_ || target == cap));
    const auto gs = atls_stream::record_batches(n, target, [&](size_t r) { return wire[r]; });
    CHECK(gs.front() == 0 && gs.back() == n);
    std::vector<size_t> wpre(n + 1, 0);
    for (size_t r = 0; r < n; r++) wpre[r + 1] = wpre[r] + wire[r];
    for (size_t k = 0; k + 1 < gs.size(); k++) {
      const size_t r0 = gs[k], r1 = gs[k + 1];
      if (n == 0) break;
      CHECK(r0 < r1);
      const size_t bytes = wpre[r1] - wpre[r0];
      CHECK(r1 == r0 + 1 || bytes <= target);
      if (r1 < n) CHECK(bytes + wire[r1] > target);
      // the connections a sender sends from this batch
      const size_t w0 = wpre[r0], w1 = wpre[r1];
      const auto cr = atls_stream::connections_in(base, w0, w1);
      for (size_t c = 0; c < nc; c++) {
        const bool overlaps = std::max(base[c], w0) < std::min(base[c + 1], w1);
        const bool in = c >= cr.first && c < cr.second;
        CHECK(!overlaps || in);                             // every connection with bytes in the batch
        CHECK(!in || overlaps || base[c + 1] == base[c]);   // and otherwise only empty ones
      }
    }
  }
  std::printf("OK\n");
  return 0;
}
