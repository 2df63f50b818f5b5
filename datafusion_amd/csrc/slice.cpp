// Sliced arrow arrays at the boundary (dfmi_column.offset, include/dfmi.h).
//
// arrow 0.12's ArrayData carries an offset: a sliced array's logical row i is
// physical slot offset + i, and value(i) / get_string(i) / is_null(i) read it
// there (/root/reference/src/execution/filter.rs:88-89,99-100). The kernels
// read offset-0 columns, so every entry point first rewrites a batch whose
// columns have offsets: fixed-width values and Utf8 offsets by pointer
// arithmetic (their slots stay aligned to their width), bitmaps (validity,
// Boolean values) by pointer when the offset keeps them 8-byte aligned, else
// as a bit-shifted copy -- on the device (k_shift_bits, on the call's stream)
// for device batches, on the host for host batches. The copies live until
// the call that made them returns (every entry point synchronises first).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "dfmi_program.h"
#include "jit.h"
#include "slice.h"

namespace dfmi {
hipError_t launch_shift_bits(const uint8_t* src, long long bit0, long long nbits, uint8_t* dst, hipStream_t st);

namespace {
int width(int t) {
    switch (t) {
        case DFMI_TYPE_INT8: case DFMI_TYPE_UINT8: return 1;
        case DFMI_TYPE_INT16: case DFMI_TYPE_UINT16: return 2;
        case DFMI_TYPE_INT32: case DFMI_TYPE_UINT32: case DFMI_TYPE_FLOAT32: return 4;
        case DFMI_TYPE_INT64: case DFMI_TYPE_UINT64: case DFMI_TYPE_FLOAT64: return 8;
        default: return 0;
    }
}

void host_shift(const uint8_t* src, int64_t bit0, int64_t nbits, uint8_t* dst) {
    const int64_t nw = (nbits + 63) / 64, src_bytes = (bit0 + nbits + 7) / 8;
    for (int64_t i = 0; i < nw; ++i) {
        const int64_t b = bit0 + i * 64, byte = b >> 3;
        const int sh = (int)(b & 7);
        uint64_t lo = 0, hi = 0;
        for (int k = 0; k < 8; ++k)
            if (byte + k < src_bytes) lo |= (uint64_t)src[byte + k] << (8 * k);
        if (sh && byte + 8 < src_bytes) hi = src[byte + 8];
        const uint64_t w = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
        memcpy(dst + i * 8, &w, 8);
    }
}
}  // namespace

Unsliced::~Unsliced() {
    for (void* p : dev) (void)hipFree(p);
}

bool any_offset(const dfmi_batch* ins, int32_t nb) {
    for (int32_t b = 0; b < nb; ++b)
        for (int i = 0; i < ins[b].num_columns; ++i)
            if (ins[b].columns && ins[b].columns[i].offset) return true;
    return false;
}

const dfmi_batch* unslice(const dfmi_batch* ins, int32_t nb, Unsliced& u, bool device, hipStream_t st) {
    size_t ncols = 0;
    for (int32_t b = 0; b < nb; ++b) ncols += (size_t)std::max(0, ins[b].num_columns);
    u.cols.resize(ncols);
    u.batches.assign(ins, ins + nb);
    size_t k = 0;
    auto bitmap = [&](const uint8_t* p, int64_t off, int64_t n) -> const uint8_t* {
        if (!p || !off) return p;
        const uint8_t* q = p + off / 8;
        if (off % 8 == 0 && ((uintptr_t)q & 7) == 0) return q;
        const size_t bytes = (size_t)((n + 63) / 64 * 8 + 8);
        if (device) {
            void* d = nullptr;
            if (hipMalloc(&d, bytes) != hipSuccess) throw Fail{DFMI_ERR_DEVICE, "hipMalloc (sliced bitmap)"};
            u.dev.push_back(d);
            if (n && launch_shift_bits(p, off, n, (uint8_t*)d, st) != hipSuccess)
                throw Fail{DFMI_ERR_DEVICE, "k_shift_bits launch failed"};
            return (const uint8_t*)d;
        }
        u.host.emplace_back(bytes, 0);
        if (n) host_shift(p, off, n, u.host.back().data());
        return u.host.back().data();
    };
    for (int32_t b = 0; b < nb; ++b) {
        const dfmi_batch& in = ins[b];
        dfmi_column* out = u.cols.data() + k;
        for (int i = 0; i < in.num_columns; ++i) {
            dfmi_column c = in.columns[i];
            const int64_t off = c.offset;
            if (off < 0) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "negative array offset"};
            if (off) {
                c.validity = bitmap(c.validity, off, c.length);
                if (c.type == DFMI_TYPE_UTF8) {
                    if (c.offsets) c.offsets += off;
                } else if (c.type == DFMI_TYPE_BOOLEAN) {
                    c.values = bitmap((const uint8_t*)c.values, off, c.length);
                } else if (c.values) {
                    c.values = (const uint8_t*)c.values + off * width(c.type);
                }
                c.offset = 0;
            }
            out[i] = c;
        }
        u.batches[b].columns = out;
        k += (size_t)std::max(0, in.num_columns);
    }
    return u.batches.data();
}
}  // namespace dfmi
