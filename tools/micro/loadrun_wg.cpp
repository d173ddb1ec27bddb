// loadrun_wg: launch coop_gen.py kernels (4-wave workgroups, 1 228 of them, 1 MiB of rows each); prints GB/s.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    hipModule_t mod;
    CK(hipModuleLoad(&mod, argv[1]));
    const size_t blk = 1024 * 1200, nblk = 1024, grid = 1228;
    void *src, *out;
    CK(hipMalloc(&src, blk * nblk + 4096));
    CK(hipMemset(src, 1, blk * nblk));
    CK(hipMalloc(&out, grid * 1024));
    struct { void* s; void* o; } args{src, out};
    size_t sz = sizeof(args);
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int k = 2; k < argc; ++k) {
        hipFunction_t f;
        CK(hipModuleGetFunction(&f, mod, argv[k]));
        for (int w = 0; w < 2; ++w) CK(hipModuleLaunchKernel(f, grid, 1, 1, 256, 1, 1, 0, nullptr, nullptr, cfg));
        CK(hipDeviceSynchronize());
        const int reps = 5;
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) CK(hipModuleLaunchKernel(f, grid, 1, 1, 256, 1, 1, 0, nullptr, nullptr, cfg));
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        std::printf("%s %.4f ms %.1f GB/s\n", argv[k], ms, (double)grid * 1024 * 1024 / (ms * 1e6));
    }
    return 0;
}
