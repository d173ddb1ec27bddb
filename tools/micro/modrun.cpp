// modrun: load a code object, launch named kernels (1-wave workgroups, args {out ptr, n}), and
// print the average time per launch.  Micro-benchmark harness for tools/micro/*_gen.py.
// usage: modrun FILE.hsaco GRID kernel1 [kernel2 ...]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    hipModule_t mod;
    CK(hipModuleLoad(&mod, argv[1]));
    const unsigned grid = (unsigned)std::atoi(argv[2]);
    void* out;
    CK(hipMalloc(&out, (size_t)grid * 256 + 4096));
    struct { void* p; unsigned n; unsigned pad; } args{out, grid, 0};
    size_t sz = sizeof(args);
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int k = 3; k < argc; ++k) {
        hipFunction_t f;
        CK(hipModuleGetFunction(&f, mod, argv[k]));
        for (int w = 0; w < 2; ++w) CK(hipModuleLaunchKernel(f, grid, 1, 1, 64, 1, 1, 0, nullptr, nullptr, cfg));
        CK(hipDeviceSynchronize());
        const int reps = 5;
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) CK(hipModuleLaunchKernel(f, grid, 1, 1, 64, 1, 1, 0, nullptr, nullptr, cfg));
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        std::printf("%s grid=%u avg_ms=%.4f\n", argv[k], grid, ms / reps);
    }
    return 0;
}
