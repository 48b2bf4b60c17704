// Residency microbenchmark (tooling, not the product): how many workgroups of a given LDS size, wave count and
// VGPR allocation a gfx950 CU keeps resident.  Every workgroup spins for `us` microseconds of s_memrealtime
// (100 MHz); a grid of k * CUs workgroups then takes ceil(k / resident) spin periods.
#include <hip/hip_runtime.h>
#include <cstdint>

template <int V>
__global__ void spin_kernel(uint64_t ticks, int* sink) {
    extern __shared__ int lds[];
    if (V == 128) asm volatile("" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127");
    else asm volatile("" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31");
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int acc = 0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        acc += lds[threadIdx.x & 63];
        __builtin_amdgcn_s_sleep(2);
    }
    if (acc == 12345) sink[threadIdx.x] = acc;   // (never true: keeps the loop)
}

extern "C" float resid_run(int waves, int lds_bytes, int vgprs, int wgs, float us) {
    int* sink = nullptr;
    if (hipMalloc(&sink, 4096) != hipSuccess) return -1.f;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const uint64_t ticks = (uint64_t)(us * 100.0f);
    auto go = [&]() {
        if (vgprs >= 128) {
            (void)hipFuncSetAttribute((const void*)spin_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
            hipLaunchKernelGGL(spin_kernel<128>, dim3(wgs), dim3(64 * waves), lds_bytes, 0, ticks, sink);
        } else {
            (void)hipFuncSetAttribute((const void*)spin_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
            hipLaunchKernelGGL(spin_kernel<32>, dim3(wgs), dim3(64 * waves), lds_bytes, 0, ticks, sink);
        }
    };
    go();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    go();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    const int err = (int)hipGetLastError();
    (void)hipFree(sink);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return err ? -(float)err : ms;
}
