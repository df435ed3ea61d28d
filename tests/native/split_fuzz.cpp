// TEST INFRASTRUCTURE ONLY: the socket path's record splitter (anothertls_amd/csrc/record_split.h,
// used by stream.cpp) driven the way a connection drives it -- received chunks appended to rx,
// whole records moved out -- for building under ASan / UBSan on the CPU. Input on stdin: repeated
// {u32 little-endian chunk length, chunk bytes}. Output: one line per record ("R <stream offset>
// <fragment length>"), then "E <code>" if the split stopped on a bad header, then "P <bytes left>".
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../anothertls_amd/csrc/record_split.h"

int main() {
  std::vector<uint8_t> rx, wire;
  std::vector<uint32_t> offs;
  int err = 0;
  // the in-place form stream.cpp uses (scan_records: records stay in rx2 until "opened", then compacted);
  // its record offsets must equal split_records' (checked at the end, exit 4 otherwise)
  std::vector<uint8_t> rx2;
  std::vector<uint32_t> offs2;
  std::vector<size_t> seen_split, seen_scan;
  size_t done2 = 0, base2 = 0;
  int err2 = 0;
  size_t base = 0;  // stream offset of rx[0]
  size_t reported = 0;
  for (;;) {
    uint8_t hdr[4];
    if (fread(hdr, 1, 4, stdin) != 4) break;
    const size_t n = (size_t)hdr[0] | ((size_t)hdr[1] << 8) | ((size_t)hdr[2] << 16) | ((size_t)hdr[3] << 24);
    std::vector<uint8_t> chunk(n);
    if (n && fread(chunk.data(), 1, n, stdin) != n) return 2;
    rx.insert(rx.end(), chunk.begin(), chunk.end());
    rx2.insert(rx2.end(), chunk.begin(), chunk.end());
    if (!err2) {
      done2 += atls_split::scan_records(rx2.data() + done2, rx2.size() - done2, done2, offs2, err2);
      for (uint32_t o : offs2) seen_scan.push_back(base2 + o);
      rx2.erase(rx2.begin(), rx2.begin() + (std::ptrdiff_t)done2);  // opened: keep the partial tail only
      base2 += done2;
      done2 = 0;
      offs2.clear();
    }
    if (err) continue;
    const size_t before = wire.size();
    const size_t used = atls_split::split_records(rx.data(), rx.size(), wire, offs, err);
    if (wire.size() - before != used) return 3;  // records are moved whole
    for (; reported < offs.size(); reported++) {
      const uint8_t* h = wire.data() + offs[reported];
      const size_t len = ((size_t)h[3] << 8) | h[4];
      printf("R %zu %zu\n", base + (offs[reported] - before), len);
      seen_split.push_back(base + (offs[reported] - before));
    }
    rx.erase(rx.begin(), rx.begin() + (std::ptrdiff_t)used);
    base += used;
  }
  if (seen_split != seen_scan || err != err2) return 4;
  if (err) printf("E %d\n", err);
  printf("P %zu\n", rx.size());
  return 0;
}
