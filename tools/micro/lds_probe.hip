// Micro-benchmark: cost of a workgroup with large dynamic LDS (zero-fill variants).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ void __launch_bounds__(512) probe(uint32_t nwords, uint32_t* out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t tid = threadIdx.x;
    if (MODE >= 1) {
        uint4* l4 = reinterpret_cast<uint4*>(lds);
        for (uint32_t i = tid; i < nwords / 4; i += 512) l4[i] = make_uint4(0, 0, 0, 0);
    }
    if (MODE == 2) {
        for (uint32_t i = tid; i < nwords; i += 512) lds[i] = 0;
    }
    __syncthreads();
    if (tid == 0 && lds[(blockIdx.x * 7) % (nwords ? nwords : 1)] == 12345) out[0] = 1;
}

int main() {
    uint32_t* out;
    (void)hipMalloc(&out, 4);
    (void)hipFuncSetAttribute((const void*)probe<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)probe<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)probe<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const uint32_t sizes[] = {16 * 1024, 48 * 1024, 64 * 1024, 80 * 1024, 100 * 1024, 152 * 1024};
    for (int mode = 0; mode < 3; ++mode)
        for (uint32_t bytes : sizes) {
            const uint32_t nw = bytes / 4;
            auto run = [&]() {
                if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(10240), dim3(512), bytes, 0, nw, out);
                if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(10240), dim3(512), bytes, 0, nw, out);
                if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(10240), dim3(512), bytes, 0, nw, out);
            };
            run();
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0, 0);
            for (int i = 0; i < 5; ++i) run();
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            std::printf("mode %d lds %6u B: %.3f ms per 10240-WG launch (err=%s)\n", mode, bytes, ms / 5,
                        hipGetErrorString(hipGetLastError()));
        }
    return 0;
}
