// Streaming-bandwidth ceiling on this MI355X: read R f64 columns, write W
// f64 columns (W <= R), with 8-byte or 16-byte lanes. Gives the achievable
// HBM rate the fused kernel is compared against (DESIGN.md "Roofline").
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

template <int R, int W, int V, int UNROLL>
__global__ __launch_bounds__(256) void stream(const double* const* in, double* const* out, long n) {
    typedef double vec __attribute__((ext_vector_type(V)));
    const long nv = n / V;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride * UNROLL) {
        vec v[UNROLL][R];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                long j = i + u * stride;
                v[u][r] = j < nv ? ((const vec*)in[r])[j] : vec(0);
            }
        if (W == 0) {
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                vec x = v[u][0];
                for (int r = 1; r < R; ++r) x += v[u][r];
                if (x[0] == -1.0) ((vec*)out[0])[i] = x;  // never true; keeps the loads
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int w = 0; w < W; ++w) {
                long j = i + u * stride;
                vec x = v[u][w];
                for (int r = W; r < R; ++r) x += v[u][r];
                if (j < nv) ((vec*)out[w])[j] = x;
            }
    }
}

template <int R, int W, int V, int U>
void run(const char* name, double** d_in, double** d_out, long n, int grid) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((stream<R, W, V, U>), dim3(grid), dim3(256), 0, 0, d_in, d_out, n);
    CHECK(hipDeviceSynchronize());
    const int reps = 10;
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((stream<R, W, V, U>), dim3(grid), dim3(256), 0, 0, d_in, d_out, n);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    double bytes = (double)n * 8 * (R + W);
    printf("%-28s grid=%6d  %8.3f ms  %7.1f GB/s\n", name, grid, ms, bytes / ms / 1e6);
}

int main(int argc, char** argv) {
    long n = argc > 1 ? atol(argv[1]) : 1000000000L;
    std::vector<double*> hin(3), hout(3);
    for (int i = 0; i < 3; ++i) {
        CHECK(hipMalloc(&hin[i], n * 8));
        CHECK(hipMalloc(&hout[i], n * 8));
        CHECK(hipMemset(hin[i], 0x3f, n * 8));
    }
    double **d_in, **d_out;
    CHECK(hipMalloc(&d_in, 3 * sizeof(double*)));
    CHECK(hipMalloc(&d_out, 3 * sizeof(double*)));
    CHECK(hipMemcpy(d_in, hin.data(), 3 * sizeof(double*), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_out, hout.data(), 3 * sizeof(double*), hipMemcpyHostToDevice));
    for (int grid : {2048, 8192, 32768}) {
        run<3, 3, 1, 4>("read3 write3 8B/lane", d_in, d_out, n, grid);
        run<3, 3, 2, 2>("read3 write3 16B/lane", d_in, d_out, n, grid);
        run<3, 0, 2, 2>("read3 16B/lane", d_in, d_out, n, grid);
        run<3, 0, 1, 4>("read3 8B/lane", d_in, d_out, n, grid);
        run<1, 1, 2, 4>("copy 16B/lane", d_in, d_out, n, grid);
    }
    return 0;
}
