// Engine internals shared by the C++ translation units of libatls.so (not part of the C ABI).
#pragma once
#include <cstdint>

#include "../../include/atls.h"

namespace atls {
// Number of installed key slots (the table every descriptor's key_slot must index).
uint32_t engine_slots(atls_engine* e);

// Held by every entry point that launches work of its own, from before its first launch until it returns: it
// stops the process's resident single-call server (ATLS_SINGLE_RESIDENT) if one runs, and no call relaunches
// the server while any hold is live -- a running server holds a hardware queue, so a kernel enqueued behind it
// would wait for its idle timeout (engine.cpp, "the resident single-call server").
struct ResidentHold {
  bool active;
  ResidentHold();
  ~ResidentHold();
  ResidentHold(const ResidentHold&) = delete;
  ResidentHold& operator=(const ResidentHold&) = delete;
};
}  // namespace atls
