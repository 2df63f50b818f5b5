// Calibration of lane-masked 8-B loads (VERDICT r05 "next round" item 1):
// what FETCH_SIZE reports, and what the memory system can move, when a
// kernel streams one column (the predicate's) and loads a second column only
// for "selected" rows -- the access pattern of the sub-tile kernels' and the
// one-tile kernel's projection-only columns at low selectivity.
//
// Every variant reads column `a` (n doubles, 8 B per lane, coalesced) and,
// for the rows a counter-based hash selects with probability p, column `c`.
// The kernel counts, per wave-load of 64 consecutive rows, the distinct 64-B
// and 128-B segments of `c` that hold a selected row (ballot), so the true
// byte count of every launch is known exactly:
//   bytes64  = 8 n + 64 * seg64     (if the memory system moves 64-B sectors)
//   bytes128 = 8 n + 128 * seg128   (if it moves whole 128-B L2 lines)
// Variant "tile" does what the sub-tile kernels do: a 256-thread block takes
// 16,384 rows, reads `a` for all of them first (the predicate pass), then
// re-reads `a` AND reads `c` for the selected rows (the output pass) -- do the
// re-reads of `a` reach HBM or the counters?
//
// usage: membw_masked [rows=1e9]; run it under rocprofv3 --pmc FETCH_SIZE (a
// pass of its own) and --kernel-trace --stats; tools/membw_masked.py joins
// the two with the printed table (DESIGN.md §6 "Calibration").
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                      \
    do {                                                              \
        hipError_t e = (x);                                           \
        if (e != hipSuccess) {                                        \
            printf("%s line %d\n", hipGetErrorString(e), __LINE__);   \
            exit(1);                                                  \
        }                                                             \
    } while (0)

typedef unsigned long long u64;

__device__ __forceinline__ u64 mix(u64 x) {
    u64 z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// segments of 8 (64 B) and 16 (128 B) consecutive lanes holding a set bit
__device__ __forceinline__ void count_segments(u64 m, u64& s64, u64& s128) {
    for (int g = 0; g < 8; ++g) s64 += ((m >> (8 * g)) & 0xffull) != 0;
    for (int g = 0; g < 4; ++g) s128 += ((m >> (16 * g)) & 0xffffull) != 0;
}

// PM = selection probability in units of 1/1000 (template: one kernel name per
// variant in the profiler's output). PM = 0: `a` only (streaming 8 B/lane).
template <int PM>
__global__ __launch_bounds__(256) void masked_stream(const double* __restrict__ a, const double* __restrict__ c,
                                                     long n, u64* counters, double* sink) {
    const u64 thresh = (u64)((double)PM / 1000.0 * 18446744073709551615.0);
    const long stride = (long)gridDim.x * blockDim.x;
    u64 s64 = 0, s128 = 0;
    double acc = 0;
    const int lane = threadIdx.x & 63;
    for (long i0 = (long)blockIdx.x * blockDim.x; i0 < n; i0 += stride * 4) {
        double x[4];
        bool sel[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long i = i0 + u * stride + threadIdx.x;
            x[u] = i < n ? a[i] : 0.0;
            sel[u] = PM > 0 && i < n && mix((u64)i) < thresh;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long i = i0 + u * stride + threadIdx.x;
            if (PM > 0) {
                const u64 m = __ballot(sel[u]);
                if (lane == 0) count_segments(m, s64, s128);
                if (sel[u]) x[u] += c[i];
            }
            acc += x[u];
        }
    }
    if (acc == -1.0) sink[0] = acc;  // never true: keeps the loads
    if (lane == 0 && PM > 0) {
        atomicAdd(&counters[0], s64);
        atomicAdd(&counters[1], s128);
    }
}

// The sub-tile shape: 256 threads x 64 rows per block tile; pass 1 reads `a`
// for every row, pass 2 re-reads `a` and reads `c` for the selected rows.
template <int PM>
__global__ __launch_bounds__(256) void masked_tile(const double* __restrict__ a, const double* __restrict__ c, long n,
                                                   u64* counters, double* sink) {
    const u64 thresh = (u64)((double)PM / 1000.0 * 18446744073709551615.0);
    constexpr int K = 64;
    const long tile = (long)blockIdx.x * 256 * K;
    const int lane = threadIdx.x & 63;
    double acc = 0;
    u64 sel = 0;  // bit k: row tile + k*256 + tid
#pragma unroll 8
    for (int k = 0; k < K; ++k) {
        const long i = tile + k * 256 + threadIdx.x;
        const double x = i < n ? a[i] : 0.0;
        acc += x;
        if (i < n && mix((u64)i) < thresh && x >= 0.0) sel |= 1ull << k;
    }
    u64 s64 = 0, s128 = 0;
    for (int k = 0; k < K; ++k) {
        const long i = tile + k * 256 + threadIdx.x;
        const bool s = (sel >> k) & 1;
        const u64 m = __ballot(s);
        if (!m) continue;
        if (lane == 0) count_segments(m, s64, s128);
        if (s) acc += a[i] * c[i];
    }
    if (acc == -1.0) sink[0] = acc;
    if (lane == 0) {
        atomicAdd(&counters[0], s64);
        atomicAdd(&counters[1], s128);
    }
}

struct Result {
    const char* name;
    double ms, s64, s128;
};

template <typename F>
Result run(const char* name, F launch, u64* dcnt, long n) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int i = 0; i < 2; ++i) launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemset(dcnt, 0, 16));
    const int reps = 5;
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    u64 h[2];
    CHECK(hipMemcpy(h, dcnt, 16, hipMemcpyDeviceToHost));
    Result r{name, ms / reps, (double)h[0] / reps, (double)h[1] / reps};
    const double b64 = 8.0 * n + 64.0 * r.s64, b128 = 8.0 * n + 128.0 * r.s128;
    printf("%-22s %9.4f ms  seg64/row %.5f seg128/row %.5f  bytes64/row %7.4f (%6.1f GB/s)  bytes128/row %7.4f "
           "(%6.1f GB/s)\n",
           name, r.ms, r.s64 / n, r.s128 / n, b64 / n, b64 / r.ms / 1e6, b128 / n, b128 / r.ms / 1e6);
    fflush(stdout);
    return r;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? (long)atof(argv[1]) : 1000000000L;
    double *a, *c, *sink;
    u64* cnt;
    CHECK(hipMalloc(&a, n * 8));
    CHECK(hipMalloc(&c, n * 8));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMalloc(&cnt, 16));
    CHECK(hipMemset(a, 0x3f, n * 8));
    CHECK(hipMemset(c, 0x3f, n * 8));
    const int grid = 8192;
    const int tgrid = (int)((n + 256 * 64 - 1) / (256 * 64));
    printf("rows %ld, one launch reads a (8 B/row) + the selected rows' segments of c\n", n);
#define STREAM(PM) run("stream p=" #PM "/1000", [&] { hipLaunchKernelGGL(masked_stream<PM>, dim3(grid), dim3(256), 0, 0, a, c, n, cnt, sink); }, cnt, n)
#define TILE(PM) run("tile p=" #PM "/1000", [&] { hipLaunchKernelGGL(masked_tile<PM>, dim3(tgrid), dim3(256), 0, 0, a, c, n, cnt, sink); }, cnt, n)
    STREAM(0);
    STREAM(10);
    STREAM(20);
    STREAM(100);
    STREAM(500);
    STREAM(1000);
    TILE(10);
    TILE(20);
    TILE(100);
    CHECK(hipDeviceSynchronize());
    return 0;
}
