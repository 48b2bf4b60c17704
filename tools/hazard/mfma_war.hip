// Write-after-read: an LDS store of accumulator registers, then an MFMA that overwrites those registers N wait states
// later.  Does the store still write the OLD values?  tdec_tail_kernel without its 48-state pad (csrc/dec_last.hip,
// ATHD_TDEC_PAD=0) stores z[0] from a[0:3] and ~6 instructions later the last MFMA of the z[3] chain writes a[0:3]; that
// build's bf16 forward differs run to run (test_bf16_forward_reproducible, round 6: 63 / 204 outputs), the padded one
// does not.  The probe runs the store, N wait states and the MFMA inside ONE asm statement (nothing inserted by the
// compiler), with the registers as VGPRs ("v") and as AGPRs ("a"), alone and beside a kernel that keeps the LDS and
// the matrix pipes busy, and counts LDS rows holding the NEW value.
//   build: hipcc --offload-arch=gfx950 -O3 -o mfma_war mfma_war.hip      run: ./mfma_war
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(16))) float f16v;
typedef __attribute__((ext_vector_type(8))) __bf16 bf8;

template <int PAD, bool AGPR>
__global__ __launch_bounds__(256) void probe(int iters, unsigned* bad) {
    __shared__ f4 lds[256];
    const int tid = threadIdx.x;
    const unsigned off = (unsigned)(size_t)&lds[tid];
    const float a = 1.0f + (tid & 7), b = 2.0f;
    unsigned nbad = 0;
    for (int it = 0; it < iters; ++it) {
        f4 v = {1.f + tid, 2.f, 3.f, 4.f};              // the OLD value the store must write
        if constexpr (AGPR) {
            asm volatile("ds_write_b128 %1, %0\n\t"
                         "s_nop %4\n\t"
                         "v_mfma_f32_16x16x4_f32 %0, %2, %3, 0\n\t"
                         "s_waitcnt lgkmcnt(0)\n\t"
                         "s_nop 15\n\ts_nop 15\n\ts_nop 15"
                         : "+a"(v) : "v"(off), "v"(a), "v"(b), "i"(PAD > 0 ? PAD - 1 : 0) : "memory");
        } else {
            asm volatile("ds_write_b128 %1, %0\n\t"
                         "s_nop %4\n\t"
                         "v_mfma_f32_16x16x4_f32 %0, %2, %3, 0\n\t"
                         "s_waitcnt lgkmcnt(0)\n\t"
                         "s_nop 15\n\ts_nop 15\n\ts_nop 15"
                         : "+v"(v) : "v"(off), "v"(a), "v"(b), "i"(PAD > 0 ? PAD - 1 : 0) : "memory");
        }
        const f4 got = lds[tid];
        nbad += (got[0] != 1.f + tid || got[1] != 2.f || got[2] != 3.f || got[3] != 4.f) ? 1u : 0u;
        __builtin_amdgcn_wave_barrier();
    }
    if (nbad) atomicAdd(bad, nbad);
}

// contention: LDS traffic (ds_write_b128 / ds_read_b128 bursts) and back-to-back MFMAs on every SIMD
__global__ __launch_bounds__(256) void busy(int iters, float* sink) {
    __shared__ float4 buf[4096];
    f16v c0 = {};
    bf8 x;
    for (int i = 0; i < 8; ++i) x[i] = (__bf16)(0.001f * (threadIdx.x + i));
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int it = 0; it < iters; ++it) {
        for (int j = 0; j < 16; ++j) buf[(threadIdx.x + 256 * j) & 4095] = make_float4(it, j, 0.f, 1.f);
        for (int j = 0; j < 16; ++j) {
            const float4 q = buf[(threadIdx.x * 7 + 256 * j + it) & 4095];
            acc.x += q.x; acc.y += q.y;
        }
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, c0, 0, 0, 0);
    }
    float s = acc.x + acc.y;
    for (int i = 0; i < 16; ++i) s += c0[i];
    if (s == 12345.f) sink[threadIdx.x] = s;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int PAD, bool AGPR>
unsigned run(bool contended, unsigned* bad, float* sink, hipStream_t s1, hipStream_t s2) {
    CK(hipMemset(bad, 0, 4));
    CK(hipDeviceSynchronize());
    if (contended) hipLaunchKernelGGL(busy, dim3(2048), dim3(256), 0, s1, 20000, sink);
    hipLaunchKernelGGL((probe<PAD, AGPR>), dim3(512), dim3(256), 0, s2, 2000, bad);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned h = 0;
    CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
    return h;
}

int main() {
    float* sink;
    unsigned* bad;
    CK(hipMalloc(&sink, 4096)); CK(hipMalloc(&bad, 4));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    printf("lane-stores checked per run: %.0f\n", 512.0 * 256 * 2000);
    for (int c = 0; c < 2; ++c) {
        const bool con = c == 1;
        printf("%s:\n", con ? "beside an LDS + MFMA busy kernel" : "alone");
        printf("  VGPR, MFMA 1 state after the store: %u new-value rows\n", run<0, false>(con, bad, sink, s1, s2));
        printf("  VGPR, MFMA 4 states after:  %u\n", run<4, false>(con, bad, sink, s1, s2));
        printf("  VGPR, MFMA 16 states after: %u\n", run<16, false>(con, bad, sink, s1, s2));
        printf("  AGPR, MFMA 1 state after the store: %u new-value rows\n", run<0, true>(con, bad, sink, s1, s2));
        printf("  AGPR, MFMA 4 states after:  %u\n", run<4, true>(con, bad, sink, s1, s2));
        printf("  AGPR, MFMA 16 states after: %u\n", run<16, true>(con, bad, sink, s1, s2));
    }
    return 0;
}
