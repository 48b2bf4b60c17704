// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 per access width (MI355X_MICROARCH.md §HBM: only the
// 16-B-per-lane streaming read is calibrated there; "calibrate on a known byte count in your own access pattern").
// Each kernel streams exactly BYTES of a buffer far larger than the 256 MiB Infinity Cache with one access width
// (coalesced, grid-stride), so FETCH_SIZE x 1024 / BYTES is the counter's factor for that width; the store kernels
// write exactly BYTES the same way.  tools/pmc_traffic.py applies the factors per kernel from its load width mix
// (tools/load_widths.py).  Build: hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/pmc_calib
//   rocprofv3 --pmc FETCH_SIZE -- tools/pmc_calib   (then a separate pass with WRITE_SIZE)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr size_t BYTES = size_t(1) << 30;       // 1 GiB per kernel
constexpr int BLOCKS = 2048, THREADS = 256;

__device__ float wave_sum(float v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <typename V>
__global__ __launch_bounds__(THREADS) void read_kernel(const V* __restrict__ x, size_t n, float* __restrict__ sink) {
    float acc = 0.f;
    for (size_t i = (size_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (size_t)BLOCKS * THREADS) {
        const V v = x[i];
        const float* f = reinterpret_cast<const float*>(&v);
        for (int j = 0; j < (int)(sizeof(V) / 4); ++j) acc += f[j];
    }
    // one dword per workgroup (8 KB in total): negligible against the 1 GiB read
    acc = wave_sum(acc);
    if (threadIdx.x == 0) sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(THREADS) void read_u16_kernel(const uint16_t* __restrict__ x, size_t n,
                                                           float* __restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (size_t)BLOCKS * THREADS) acc += x[i];
    const float a = wave_sum((float)acc);
    if (threadIdx.x == 0) sink[blockIdx.x] = a;
}

template <typename V>
__global__ __launch_bounds__(THREADS) void write_kernel(V* __restrict__ y, size_t n) {
    V v;
    float* f = reinterpret_cast<float*>(&v);
    for (int j = 0; j < (int)(sizeof(V) / 4); ++j) f[j] = (float)j;
    for (size_t i = (size_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (size_t)BLOCKS * THREADS) y[i] = v;
}

__global__ __launch_bounds__(THREADS) void write_u16_kernel(uint16_t* __restrict__ y, size_t n) {
    for (size_t i = (size_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (size_t)BLOCKS * THREADS)
        y[i] = (uint16_t)i;
}

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main() {
    void* buf = nullptr;
    float* sink = nullptr;
    CHECK(hipMalloc(&buf, BYTES));
    CHECK(hipMalloc(&sink, BLOCKS * sizeof(float)));
    CHECK(hipMemset(buf, 0, BYTES));
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(read_u16_kernel, dim3(BLOCKS), dim3(THREADS), 0, 0, (const uint16_t*)buf, BYTES / 2, sink);
        hipLaunchKernelGGL(read_kernel<float>, dim3(BLOCKS), dim3(THREADS), 0, 0, (const float*)buf, BYTES / 4, sink);
        hipLaunchKernelGGL(read_kernel<float2>, dim3(BLOCKS), dim3(THREADS), 0, 0, (const float2*)buf, BYTES / 8, sink);
        hipLaunchKernelGGL(read_kernel<float4>, dim3(BLOCKS), dim3(THREADS), 0, 0, (const float4*)buf, BYTES / 16, sink);
        hipLaunchKernelGGL(write_u16_kernel, dim3(BLOCKS), dim3(THREADS), 0, 0, (uint16_t*)buf, BYTES / 2);
        hipLaunchKernelGGL(write_kernel<float>, dim3(BLOCKS), dim3(THREADS), 0, 0, (float*)buf, BYTES / 4);
        hipLaunchKernelGGL(write_kernel<float2>, dim3(BLOCKS), dim3(THREADS), 0, 0, (float2*)buf, BYTES / 8);
        hipLaunchKernelGGL(write_kernel<float4>, dim3(BLOCKS), dim3(THREADS), 0, 0, (float4*)buf, BYTES / 16);
    }
    CHECK(hipDeviceSynchronize());
    printf("pmc_calib: %zu bytes per kernel, 2 repetitions\n", BYTES);
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
