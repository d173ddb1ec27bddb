// Host-only ASan/UBSan driver (race detection / sanitizers): the column-program
// compiler (rq_colprog.cpp: elimination + IR), its allocator, emitter and machine emulator
// (rq_colasm.cpp), the CPU port (rq_cpu.cpp) and the fecquic wire/ring code, exercised under
// -fsanitize=address,undefined.  Checks emulated machine programs and the CPU port against the IR's
// own host evaluation on random blocks.  Built and run by tests/test_sanitize.py (`make sanitize`).
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../rl-quic-raptor_amd/csrc/rq_colasm.hpp"
#include "../../rl-quic-raptor_amd/csrc/rq_colprog.hpp"
#include "../../rl-quic-raptor_amd/fecquic/fq_wire.hpp"

extern "C" int rqc_encode(uint32_t K, uint32_t T, uint32_t n_blocks, const uint8_t* src, uint64_t src_stride,
                          const uint32_t* esi, uint32_t n_esi, uint8_t* out, uint64_t out_stride, int threads);

using namespace rq;

int main() {
    std::mt19937_64 rng(7);
    int bad = 0;
    for (uint32_t K : {1u, 10u, 26u, 64u, 256u, 1024u}) {
        Params p;
        params_for_K(K, &p);
        const uint32_t T = 64, R = K / 8 + 9;
        std::vector<uint32_t> esi;
        for (uint32_t i = 0; i < R; ++i) esi.push_back(K + i * (i % 3 ? 1 : 7));
        esi.push_back(3 % K);  // a source row among the outputs
        std::vector<uint8_t> src((size_t)K * T);
        for (auto& b : src) b = (uint8_t)rng();
        ColIR ir;
        std::string err;
        if (!build_colprog(p, esi.data(), (uint32_t)esi.size(), &ir, &err)) { std::printf("build %u: %s\n", K, err.c_str()); return 1; }
        std::vector<uint8_t> ref(esi.size() * T), emu(esi.size() * T), cpu(esi.size() * T);
        eval_colprog(ir, src.data(), T, ref.data());
        for (uint32_t nl : {0u, 40u, 156u}) {  // register-only, small and default LDS spill tiers
            AllocOpts o;
            o.n_lds = nl;
            if (K >= 256) o.n_vgpr = 120;  // force global scratch traffic too
            MProg mp;
            if (!allocate_colprog(ir, o, &mp, &err)) { std::printf("alloc %u: %s\n", K, err.c_str()); return 1; }
            std::fill(emu.begin(), emu.end(), 0);
            if (!emulate_colprog(mp, src.data(), T, emu.data(), &err)) { std::printf("emulate %u: %s\n", K, err.c_str()); return 1; }
            const std::string a = emit_colprog_asm(mp, "k");
            bad += emu != ref || a.empty();
        }
        if (rqc_encode(K, T, 1, src.data(), src.size(), esi.data(), (uint32_t)esi.size(), cpu.data(), cpu.size(), 2))
            return 1;
        bad += cpu != ref;
        std::printf("K=%u nodes=%zu ok=%d\n", K, ir.nodes.size(), bad == 0);
    }
    uint8_t b[fq::HEADER_MAX_LEN];
    fq::FecHeader h, g;
    h.block_id = 70000; h.n = 2260; h.k = 2048; h.sym_id = 2259; h.payload_len = 1200;
    bad += fq::marshal_auto(h, b) != fq::HEADER_V2_LEN || !fq::unmarshal(b, sizeof b, &g) || g.k != 2048;
    std::printf(bad ? "FAIL %d\n" : "ALL OK\n", bad);
    return bad != 0;
}
