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
constexpr uint8_t kValNum = 8u;        // number / boolean / NaN: `v += undefined` is NaN (combine "incr")
constexpr uint8_t kValNever = 16u;     // matches nothing, itself included (NaN; a consensus {value: undefined})
constexpr uint8_t kValSeqM1 = 32u;
constexpr uint32_t kValueCombineFail = 0xFFFFFFFEu;  // result slot: combine unsupported here (device: MT_UNSUPPORTED)     // an object with own seq === -1: consensus would update it in place

// values: JSON texts (index 0 = null); flags: one per value (kValFalsy and kValNever / kValNum of
// derived values set by the caller).  Out: cls[v] structural class (equal classes match),
// flags |= kValIrregular / kValUnknown / kValNum / kValSeqM1, exc = sorted (u << 32 | v) pairs
// with R(u, v) and different classes.  kValNever values get classes of their own and no
// exceptions.  Returns 1 when the pairwise pass was skipped (more than max_pairs pairs).
int value_relations(const std::vector<std::string> &values, std::vector<uint32_t> &cls, std::vector<uint8_t> &flags,
                    std::vector<uint64_t> &exc, int64_t max_pairs = 50000000);

// Properties.combine(combiningInfo, undefined, undefined, seq) (properties.ts:26-60) — the value a
// key gets from an annotate with a combiningOp when the segment does not have the key
// (segmentPropertiesManager.ts:93-98: previousValue undefined, newValue undefined).  def / min:
// JSON texts of defaultValue / minValue, null when undefined.  Writes the result's JSON text to
// `out` where there is one.
enum CombineResult {
    kCombineValue,        // an ordinary value: `out`
    kCombineMin,          // minValue itself (the clamp of "incr")
    kCombineNaN,          // NaN ("incr" of a number / boolean / undefined / null)
    kCombineConsensus,    // a new { value: undefined, seq } (JSON text `out`): matches nothing
    kCombineDelete,       // null: the key stays absent
    kCombineUnsupported   // the key would hold undefined, or combine throws
};
CombineResult combine_absent(int kind, const std::string *def, const std::string *min, int32_t seq, std::string &out);

// String(v) of a value given as JSON text (an object key: idToSegment[id], mergeTree.ts:1185);
// false when the text does not parse
bool js_string_of(const std::string &json, std::u16string &out);

// JSON.stringify helpers shared with mt_json.cpp
void json_quote(std::string &o, const char16_t *s, size_t n);
void json_number(std::string &o, double v);

}  // namespace mt
