// Fixed gfx950 kernels of libdfmi (the query kernels themselves are generated
// and compiled per query shape by jit.cpp over jit_skeleton.hip):
//
//   k_pack_bools       byte-per-row -> LSB-first bitmap for Boolean outputs of
//                      a filtered projection (the compacted row count is only
//                      known on the device, so the packing is a second pass).
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

hipError_t launch_gen_unit_f64(u64 key, i64 row0, i64 n, double* out, hipStream_t st) {
    hipLaunchKernelGGL(k_gen_unit_f64, dim3(8192), dim3(256), 0, st, key, row0, n, out);
    return hipGetLastError();
}

hipError_t launch_gen_i64(u64 key, i64 row0, i64 n, i64 lo, u64 range, i64* out, hipStream_t st) {
    hipLaunchKernelGGL(k_gen_i64, dim3(8192), dim3(256), 0, st, key, row0, n, lo, range, out);
    return hipGetLastError();
}
}  // namespace dfmi
