// Does an LDS store that reads a v_mfma_f32_16x16x4_f32 result N wait states after the MFMA see the result, on
// gfx950, alone and with another kernel's MFMAs sharing the SIMDs?  (the tdec_tail_kernel pad,
// csrc/dec_last.hip.)  hipcc pads such a store with `s_nop 8` (9 wait states, tools/hazard/README.md); the probe
// issues the MFMA, exactly N wait states of s_nop and the ds_write_b128 inside ONE asm statement (the compiler
// inserts nothing inside it), with the destination registers preset to a sentinel, then checks what reached LDS.
//   build: hipcc --offload-arch=gfx950 -O3 -o mfma_ds mfma_ds.hip      run: ./mfma_ds
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(16))) float f16v;
typedef __attribute__((ext_vector_type(8))) __bf16 bf8;


template <int PAD>
__device__ __forceinline__ f4 mfma_then_store(float a, float b, void* lds_addr_dummy, unsigned lds_off) {
    f4 acc = {-7.f, -7.f, -7.f, -7.f};                  // sentinel: what a stale read of the destination returns
    if constexpr (PAD == 0) {
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, 0\n\t"
                     "ds_write_b128 %3, %0\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "+v"(acc) : "v"(a), "v"(b), "v"(lds_off) : "memory");
    } else {
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, 0\n\t"
                     "s_nop %4\n\t"
                     "ds_write_b128 %3, %0\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "+v"(acc) : "v"(a), "v"(b), "v"(lds_off), "i"(PAD - 1) : "memory");
    }
    return acc;
}

// the same after a chain of 12 dependent MFMAs (tdec_tail_kernel's form: the last of a 12-MFMA accumulation chain is
// followed by the store), the chain's first MFMA starting from 0
template <int PAD>
__device__ __forceinline__ void chain_then_store(float a, float b, unsigned lds_off) {
    f4 acc = {-7.f, -7.f, -7.f, -7.f};
    asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, 0\n\t"
                 ".rept 11\n\t"
                 "v_mfma_f32_16x16x4_f32 %0, %1, %2, %0\n\t"
                 ".endr\n\t"
                 "s_nop %4\n\t"
                 "ds_write_b128 %3, %0\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "+v"(acc) : "v"(a), "v"(b), "v"(lds_off), "i"(PAD - 1) : "memory");
}
template <int PAD>
__global__ __launch_bounds__(256) void probe_chain(const float* av, const float* bv, int iters, unsigned* bad) {
    __shared__ f4 lds[256];
    const int tid = threadIdx.x;
    const unsigned off = (unsigned)(size_t)&lds[tid];
    const float a = av[(blockIdx.x * 256 + tid) & 1023], b = bv[(blockIdx.x * 256 + tid) & 1023];
    f4 ref = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 12; ++i) ref = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, ref, 0, 0, 0);
    unsigned nbad = 0;
    for (int it = 0; it < iters; ++it) {
        chain_then_store<PAD>(a, b, off);
        const f4 got = lds[tid];
        nbad += (got[0] != ref[0] || got[1] != ref[1] || got[2] != ref[2] || got[3] != ref[3]) ? 1u : 0u;
        __builtin_amdgcn_wave_barrier();
    }
    if (nbad) atomicAdd(bad, nbad);
}

// probe: every lane's four MFMA outputs as stored to LDS vs the reference (computed with a 48-state pad, then
// checked equal to the compiler-padded builtin); counts mismatching lanes
template <int PAD>
__global__ __launch_bounds__(256) void probe(const float* av, const float* bv, int iters, unsigned* bad) {
    __shared__ f4 lds[256];
    const int tid = threadIdx.x;
    const unsigned off = (unsigned)(size_t)&lds[tid];   // (LDS address: the low 32 bits of the shared pointer)
    const float a = av[(blockIdx.x * 256 + tid) & 1023], b = bv[(blockIdx.x * 256 + tid) & 1023];
    f4 ref = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, (f4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    unsigned nbad = 0;
    for (int it = 0; it < iters; ++it) {
        mfma_then_store<PAD>(a, b, nullptr, off);
        const f4 got = lds[tid];
        nbad += (got[0] != ref[0] || got[1] != ref[1] || got[2] != ref[2] || got[3] != ref[3]) ? 1u : 0u;
        __builtin_amdgcn_wave_barrier();
    }
    if (nbad) atomicAdd(bad, nbad);
}

// contention: back-to-back 32x32x16 bf16 MFMAs on every SIMD (independent accumulators), ~spin ms
__global__ __launch_bounds__(256) void busy(int iters, float* sink) {
    f16v c0 = {}, c1 = {}, c2 = {}, c3 = {};
    bf8 x;
    for (int i = 0; i < 8; ++i) x[i] = (__bf16)(0.001f * (threadIdx.x + i));
    for (int it = 0; it < iters; ++it) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, c3, 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
    if (s == 12345.f) sink[threadIdx.x] = s;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int PAD>
unsigned run_chain(bool contended, const float* a, const float* b, unsigned* bad, float* sink, hipStream_t s1,
                   hipStream_t s2) {
    CK(hipMemset(bad, 0, 4));
    CK(hipDeviceSynchronize());
    if (contended) hipLaunchKernelGGL(busy, dim3(1024), dim3(256), 0, s1, 200000, sink);
    hipLaunchKernelGGL(probe_chain<PAD>, dim3(512), dim3(256), 0, s2, a, b, 500, bad);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned h = 0;
    CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
    return h;
}

template <int PAD>
unsigned run(bool contended, const float* a, const float* b, unsigned* bad, float* sink, hipStream_t s1, hipStream_t s2) {
    CK(hipMemset(bad, 0, 4));
    CK(hipDeviceSynchronize());
    if (contended) hipLaunchKernelGGL(busy, dim3(1024), dim3(256), 0, s1, 200000, sink);
    hipLaunchKernelGGL(probe<PAD>, dim3(512), dim3(256), 0, s2, a, b, 2000, bad);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned h = 0;
    CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
    return h;
}

int main() {
    std::vector<float> h(1024);
    for (int i = 0; i < 1024; ++i) h[i] = 0.25f + (float)((i * 37) % 101) / 64.f;
    float *a, *b, *sink;
    unsigned* bad;
    CK(hipMalloc(&a, 4096)); CK(hipMalloc(&b, 4096)); CK(hipMalloc(&sink, 4096)); CK(hipMalloc(&bad, 4));
    CK(hipMemcpy(a, h.data(), 4096, hipMemcpyHostToDevice));
    for (int i = 0; i < 1024; ++i) h[i] = 1.5f - (float)((i * 53) % 97) / 80.f;
    CK(hipMemcpy(b, h.data(), 4096, hipMemcpyHostToDevice));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const double checks = 512.0 * 256 * 2000;
    printf("lane-stores checked per run: %.0f\n", checks);
    for (int c = 0; c < 2; ++c) {
        const bool con = c == 1;
        printf("%s:\n", con ? "with a concurrent MFMA kernel" : "alone");
        printf("  pad  0 wait states: %u mismatches\n", run<0>(con, a, b, bad, sink, s1, s2));
        printf("  pad  4 wait states: %u mismatches\n", run<4>(con, a, b, bad, sink, s1, s2));
        printf("  pad  9 wait states (hipcc's s_nop 8): %u mismatches\n", run<9>(con, a, b, bad, sink, s1, s2));
        printf("  pad 10 wait states: %u mismatches\n", run<10>(con, a, b, bad, sink, s1, s2));
        printf("  pad 16 wait states: %u mismatches\n", run<16>(con, a, b, bad, sink, s1, s2));
        printf("  12-MFMA chain, pad  4: %u mismatches (of %.0f)\n", run_chain<4>(con, a, b, bad, sink, s1, s2), checks / 4);
        printf("  12-MFMA chain, pad  9 (hipcc's s_nop 8): %u mismatches\n", run_chain<9>(con, a, b, bad, sink, s1, s2));
        printf("  12-MFMA chain, pad 10: %u mismatches\n", run_chain<10>(con, a, b, bad, sink, s1, s2));
        printf("  12-MFMA chain, pad 16: %u mismatches\n", run_chain<16>(con, a, b, bad, sink, s1, s2));
    }
    return 0;
}
