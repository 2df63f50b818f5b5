// Fixed gfx950 kernels of libdfmi (the query kernels themselves are generated
// and compiled per query shape by jit.cpp over jit_skeleton.hip):
//
//   k_pack_bools       byte-per-row -> LSB-first bitmap for Boolean outputs of
//                      a filtered projection (the compacted row count is only
//                      known on the device, so the packing is a second pass).
//   k_utf8_copy_rows   second pass of the two-pass Utf8 gather: the bytes of
//                      the compacted rows, from the offsets / source starts
//                      the query kernel wrote.
//   k_gen_*            counter-based synthetic columns (bench / test inputs,
//                      include/dfmi_datasource.h).
//   k_rebase_offsets / k_place_bits
//                      the root's side of dfmi_shard_gather_to_root: a rank's
//                      Utf8 offsets moved to its global byte base, a rank's
//                      bitmap ORed in at its global row offset.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace dfmi {

typedef unsigned long long u64;
typedef long long i64;

// Boolean outputs of a filtered projection: one byte per row -> bitmap.
__global__ void k_pack_bools(const uint8_t* bytes, uint8_t* bits, const u64* count) {
    const i64 n = (i64)*count;
    const i64 nb = (n + 7) >> 3;
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (i64)gridDim.x * blockDim.x) {
        unsigned v = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const i64 r = i * 8 + j;
            if (r < n) v |= (unsigned)(bytes[r] & 1) << j;
        }
        bits[i] = (uint8_t)v;
    }
}

// ------------------------------------------- two-pass Utf8 gather ---
// Second pass (jit Launch::gather == 3): the query kernel wrote the output
// offset (final one included) and the source start of each of the R selected
// rows; this copies their bytes. A wave owns 64 consecutive output rows, i.e.
// one contiguous output byte range, and its lanes take the range's aligned
// output words in turn: the row holding a word's first byte by binary search
// over the wave's 65 offsets in LDS; a word inside one string is assembled
// from two aligned source words (v_alignbyte), a word spanning strings byte by
// byte. Words inside the range are stored whole, the two edge words the range
// shares with the neighbouring waves bytewise. R and the byte total come from
// the kernel's totals on the device (no host round trip).
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

__global__ __launch_bounds__(256) void k_utf8_copy_rows(const int32_t* offs, const int32_t* spos, const uint8_t* src,
                                                        uint8_t* out, const u64* totals, int chan, i64 cap) {
    __shared__ int so[4][65];
    __shared__ int ss[4][64];
    const i64 R = (i64)totals[0];
    if ((i64)totals[chan] > cap) return;  // the query kernel reported the capacity error
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int* O = so[wave];
    int* S = ss[wave];
    const unsigned m = (unsigned)((uintptr_t)out & 3u);
    unsigned* ow = (unsigned*)(out - m);  // aligned frame: output byte q is frame byte q + m
    for (i64 g = (i64)blockIdx.x * 4 + wave; g * 64 < R; g += (i64)gridDim.x * 4) {
        const i64 r0 = g * 64;
        const int nr = (int)(R - r0 < 64 ? R - r0 : 64);
        wave_lds_fence();  // the previous group's reads of O / S come first
        if (lane < nr) {
            O[lane] = offs[r0 + lane];
            S[lane] = spos[r0 + lane];
        }
        if (lane == 0) O[nr] = offs[r0 + nr];
        wave_lds_fence();
        const i64 B0 = O[0], B1 = O[nr];
        if (B1 <= B0) continue;
        const i64 wend = (B1 - 1 + m) >> 2;  // last frame word holding range bytes
        for (i64 w = ((B0 + m) >> 2) + lane; w <= wend; w += 64) {
            const i64 p = 4 * w - m;  // output byte at the word's frame byte 0
            const i64 q0 = p > B0 ? p : B0, q1 = p + 4 < B1 ? p + 4 : B1;
            int lo = 0, hi = nr - 1;  // the last row starting at or before q0 (offsets non-decreasing)
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (O[mid] <= q0) lo = mid;
                else hi = mid - 1;
            }
            int r = lo;
            unsigned val;
            if (q1 <= O[r + 1]) {  // one string: source bytes [a, a + q1 - q0)
                const uintptr_t a = (uintptr_t)(src + S[r] + (q0 - O[r]));
                const unsigned* aw = (const unsigned*)(a & ~(uintptr_t)3);
                const unsigned sh = (unsigned)(a & 3u);
                const unsigned lw = aw[0];
                const unsigned hw = sh + (unsigned)(q1 - q0) > 4u ? aw[1] : 0u;
                val = __builtin_amdgcn_alignbyte(hw, lw, sh) << (8u * (unsigned)(q0 - p));
            } else {
                val = 0;
                for (i64 q = q0; q < q1; ++q) {
                    while (O[r + 1] <= q) ++r;
                    val |= (unsigned)src[S[r] + (q - O[r])] << (8u * (unsigned)(q - p));
                }
            }
            if (q0 == p && q1 == p + 4) {
                ow[w] = val;
            } else {
                for (i64 q = q0; q < q1; ++q) out[q] = (uint8_t)(val >> (8u * (unsigned)(q - p)));
            }
        }
    }
}

// ------------------------------------------------- synthetic inputs ---
__device__ __forceinline__ u64 splitmix64(u64 x) {
    u64 z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_gen_unit_f64(u64 key, i64 row0, i64 n, double* out) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x)
        out[i] = (double)(splitmix64(key ^ (u64)(row0 + i)) >> 11) * 0x1.0p-53;
}

__global__ void k_gen_i64(u64 key, i64 row0, i64 n, i64 lo, u64 range, i64* out) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x)
        out[i] = lo + (i64)(splitmix64(key ^ (u64)(row0 + i)) % range);
}

// ------------------------------------------------- shard gather (root) ---
__global__ void k_rebase_offsets(const int32_t* src, i64 n, i64 base, int32_t* dst) {
    const int32_t s0 = src[0];
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (i64)gridDim.x * blockDim.x)
        dst[i] = (int32_t)(src[i] - s0 + base);
}

// bits [0, n) of src ORed into dst at bit dst_bit (dst zeroed, 4-byte aligned).
__global__ void k_place_bits(const uint8_t* src, i64 n, unsigned* dst, i64 dst_bit) {
    const i64 nw = (n + 31) >> 5;
    for (i64 j = (i64)blockIdx.x * blockDim.x + threadIdx.x; j < nw; j += (i64)gridDim.x * blockDim.x) {
        u64 v = 0;
        for (int b = 0; b < 4; ++b) {
            const i64 byte = j * 4 + b;
            if (byte * 8 < n) v |= (u64)src[byte] << (8 * b);
        }
        const i64 rem = n - j * 32;
        if (rem < 32) v &= (1ull << rem) - 1;  // bits past n are not the source's
        if (!v) continue;
        const i64 pos = dst_bit + j * 32;
        const u64 sh = v << (pos & 31);
        atomicOr(&dst[pos >> 5], (unsigned)sh);
        if (sh >> 32) atomicOr(&dst[(pos >> 5) + 1], (unsigned)(sh >> 32));
    }
}

// ------------------------------------------- sliced arrays (slice.cpp) ---
// dst word i = bits [bit0 + 64 i, bit0 + 64 i + 64) of src (src_bytes bytes
// readable): a bitmap at an arrow array offset moved to bit 0.
__global__ void k_shift_bits(const uint8_t* src, i64 bit0, i64 src_bytes, u64* dst, i64 nwords) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (i64)gridDim.x * blockDim.x) {
        const i64 b = bit0 + i * 64, byte = b >> 3;
        const int sh = (int)(b & 7);
        u64 lo = 0, hi = 0;
        for (int k = 0; k < 8; ++k)
            if (byte + k < src_bytes) lo |= (u64)src[byte + k] << (8 * k);
        if (sh && byte + 8 < src_bytes) hi = src[byte + 8];
        dst[i] = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
    }
}

hipError_t launch_shift_bits(const uint8_t* src, i64 bit0, i64 nbits, uint8_t* dst, hipStream_t st) {
    const i64 nw = (nbits + 63) / 64;
    const int grid = (int)std::max<i64>(1, std::min<i64>((nw + 255) / 256, 4096));
    hipLaunchKernelGGL(k_shift_bits, dim3(grid), dim3(256), 0, st, src, bit0, (bit0 + nbits + 7) / 8, (u64*)dst, nw);
    return hipGetLastError();
}

hipError_t launch_rebase_offsets(const int32_t* src, i64 n, i64 base, int32_t* dst, hipStream_t st) {
    const int grid = (int)std::max<i64>(1, std::min<i64>((n + 256) / 256, 4096));
    hipLaunchKernelGGL(k_rebase_offsets, dim3(grid), dim3(256), 0, st, src, n, base, dst);
    return hipGetLastError();
}

hipError_t launch_place_bits(const uint8_t* src, i64 n, uint8_t* dst, i64 dst_bit, hipStream_t st) {
    const int grid = (int)std::max<i64>(1, std::min<i64>(((n + 31) / 32 + 255) / 256, 4096));
    hipLaunchKernelGGL(k_place_bits, dim3(grid), dim3(256), 0, st, src, n, (unsigned*)dst, dst_bit);
    return hipGetLastError();
}

hipError_t launch_pack_bools(const uint8_t* bytes, uint8_t* bits, const u64* count, i64 max_rows,
                             hipStream_t st) {
    const i64 nb = (max_rows + 7) / 8;
    int grid = (int)std::min<i64>((nb + 255) / 256, 4096);
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(k_pack_bools, dim3(grid), dim3(256), 0, st, bytes, bits, count);
    return hipGetLastError();
}

hipError_t launch_utf8_copy_rows(const int32_t* offs, const int32_t* spos, const uint8_t* src, uint8_t* out,
                                 const u64* totals, int chan, i64 cap, i64 max_rows, hipStream_t st) {
    const int grid = (int)std::max<i64>(1, std::min<i64>((max_rows + 255) / 256, 8192));
    hipLaunchKernelGGL(k_utf8_copy_rows, dim3(grid), dim3(256), 0, st, offs, spos, src, out, totals, chan, cap);
    return hipGetLastError();
}

hipError_t launch_gen_unit_f64(u64 key, i64 row0, i64 n, double* out, hipStream_t st) {
    hipLaunchKernelGGL(k_gen_unit_f64, dim3(8192), dim3(256), 0, st, key, row0, n, out);
    return hipGetLastError();
}

hipError_t launch_gen_i64(u64 key, i64 row0, i64 n, i64 lo, u64 range, i64* out, hipStream_t st) {
    hipLaunchKernelGGL(k_gen_i64, dim3(8192), dim3(256), 0, st, key, row0, n, lo, range, out);
    return hipGetLastError();
}
}  // namespace dfmi
