// Sliced arrow arrays at the boundary (slice.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/dfmi.h"

namespace dfmi {
// Offset-0 copies of a call's batch descriptors (and any shifted bitmaps).
struct Unsliced {
    std::vector<dfmi_column> cols;
    std::vector<dfmi_batch> batches;
    std::vector<void*> dev;                   // shifted device bitmaps
    std::vector<std::vector<uint8_t>> host;   // shifted host bitmaps
    ~Unsliced();
};
bool any_offset(const dfmi_batch* ins, int32_t nb);
// `ins` with every column at offset 0; device bitmaps shifted on `st`.
const dfmi_batch* unslice(const dfmi_batch* ins, int32_t nb, Unsliced& u, bool device, hipStream_t st);
}  // namespace dfmi
