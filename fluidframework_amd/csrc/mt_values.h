// mt_values.h — structural matchProperties classes of interned property values (mt_values.cpp).
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

namespace mt {

// per-value flags (mt_batch value_flags; bit 0, JS-falsy, is set by the caller)
constexpr uint8_t kValFalsy = 1u;
constexpr uint8_t kValIrregular = 2u;  // in at least one exception pair (see mt_values.cpp)
constexpr uint8_t kValUnknown = 4u;    // pairwise pass skipped: class-different comparisons are unsupported

// values: JSON texts (index 0 = null).  Out: cls[v] structural class (equal classes match),
// flags |= kValIrregular / kValUnknown, exc = sorted (u << 32 | v) pairs with R(u, v) and
// different classes.  Returns 1 when the pairwise pass was skipped (more than max_pairs pairs).
int value_relations(const std::vector<std::string> &values, std::vector<uint32_t> &cls, std::vector<uint8_t> &flags,
                    std::vector<uint64_t> &exc, int64_t max_pairs = 50000000);

}  // namespace mt
