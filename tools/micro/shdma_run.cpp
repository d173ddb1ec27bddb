// shdma_run: clockrun with REPS / WARM launches per kernel (tools/micro/shdma_gen.py); hipcc -O2 --offload-arch=gfx950 tools/micro/shdma_run.cpp -o tools/micro/shdma_run
// one wave per workgroup, 5 waves per block (5120 workgroups); prints ms and GB/s per kernel.
// hipcc -O2 --offload-arch=gfx950 tools/micro/clockrun.cpp -o tools/micro/clockrun
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    hipModule_t mod;
    CK(hipModuleLoad(&mod, argv[1]));
    const size_t blk = 1024 * 1200, nblk = 1024, grid = argc > 0 && getenv("GRID") ? atoi(getenv("GRID")) : nblk * 5;
    void *src, *out;
    CK(hipMalloc(&src, blk * nblk + 4096));
    {
        std::vector<uint32_t> h((blk * nblk + 4096) / 4);
        uint64_t x = 88172645463325252ull;
        for (auto& w : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; w = (uint32_t)x; }
        CK(hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
    CK(hipMalloc(&out, grid * 1024));
    const unsigned wgs = getenv("WGS") ? atoi(getenv("WGS")) : 64;
    struct { void* s; void* o; } args{src, out};
    size_t sz = sizeof(args);
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int k = 2; k < argc; ++k) {
        hipFunction_t f;
        CK(hipModuleGetFunction(&f, mod, argv[k]));
        for (int w = 0; w < (getenv("WARM") ? atoi(getenv("WARM")) : 2); ++w) CK(hipModuleLaunchKernel(f, grid, 1, 1, wgs, 1, 1, 0, nullptr, nullptr, cfg));
        CK(hipDeviceSynchronize());
        const int reps = getenv("REPS") ? atoi(getenv("REPS")) : 5;
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) CK(hipModuleLaunchKernel(f, grid, 1, 1, wgs, 1, 1, 0, nullptr, nullptr, cfg));
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        std::printf("%s %.4f ms %.1f GB/s\n", argv[k], ms, blk * nblk / (ms * 1e6));
    }
    return 0;
}
