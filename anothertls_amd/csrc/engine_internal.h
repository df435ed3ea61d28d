// Engine internals shared by the C++ translation units of libatls.so (not part of the C ABI).
#pragma once
#include <cstdint>

#include "../../include/atls.h"

namespace atls {
// Number of installed key slots (the table every descriptor's key_slot must index).
uint32_t engine_slots(atls_engine* e);
}  // namespace atls
