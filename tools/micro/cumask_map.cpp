// cumask_map: where the workgroups of a CU-masked stream run.  For each test mask (256 bits, as
// hipExtStreamCreateWithCUMask takes it) launches 2048 one-wave workgroups and prints, per XCC, the
// number of distinct (SE, CU) pairs they reported (HW_REG_XCC_ID, HW_REG_HW_ID).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <set>
#include <utility>
#include <vector>

__global__ void where(unsigned* out) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    for (int i = 0; i < 2000; ++i) asm volatile("s_nop 7");  // keep the slot a while
    if (threadIdx.x == 0) { out[2 * blockIdx.x] = hw; out[2 * blockIdx.x + 1] = xcc; }
}

static void run(const char* name, const unsigned* mask, unsigned* d) {
    const int n = 2048;
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, 8, mask) != hipSuccess) { std::printf("%s: create failed\n", name); return; }
    hipLaunchKernelGGL(where, dim3(n), dim3(64), 0, s, d);
    if (hipStreamSynchronize(s) != hipSuccess) { std::printf("%s: sync failed\n", name); return; }
    std::vector<unsigned> h(2 * n);
    hipMemcpy(h.data(), d, 8 * n, hipMemcpyDeviceToHost);
    std::set<std::pair<unsigned, unsigned>> per[16];
    for (int i = 0; i < n; ++i) {
        const unsigned hw = h[2 * i], x = h[2 * i + 1] & 0xF;
        per[x].insert({(hw >> 13) & 7, (hw >> 8) & 0xF});
    }
    std::printf("%-22s", name);
    for (int x = 0; x < 8; ++x) std::printf(" xcc%d:%2zu", x, per[x].size());
    std::printf("\n");
    hipStreamDestroy(s);
}

int main() {
    unsigned* d;
    if (hipMalloc(&d, 2048 * 8) != hipSuccess) return 1;
    unsigned m[8];
    auto clr = [&] { for (unsigned& v : m) v = 0; };
    for (unsigned& v : m) v = 0xFFFFFFFFu;
    run("all", m, d);
    clr(); m[0] = 1; run("bit0", m, d);
    clr(); m[0] = 3; run("bits0-1", m, d);
    clr(); m[0] = 1; m[1] = 1; run("bit0+bit32", m, d);
    clr(); m[0] = 0xFFFFFFFFu; run("dword0", m, d);
    clr(); m[0] = 0xFF; run("bits0-7", m, d);
    clr(); for (int i = 0; i < 8; ++i) m[i] = 3; run("bits0-1 of each dword", m, d);
    clr(); m[0] = 0xFFFF; run("bits0-15", m, d);
    clr(); m[7] = 0x80000000u; run("bit255", m, d);
    return 0;
}
