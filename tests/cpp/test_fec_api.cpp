// C++ test of the go/fec mirror (rl-quic-raptor_amd/csrc/fec_raptorq.hpp) over librqhip.so.
// Mirrors TestRaptorQ_ExperimentB_Scaled (go/integrationtests/fec/raptorq_experiments_test.go:
// 105-310): K=5, L=1100, N=8, Bernoulli loss from a seeded PRNG, round-trip equality.
// Usage: test_fec_api cpu   -> argument/error behaviour only (no device needed)
//        test_fec_api gpu   -> full encode / lossy decode round trips on the GPU
#include <cstdio>
#include <cstring>
#include <random>

#include "fec_raptorq.hpp"

#define CHECK(c)                                                           \
    do {                                                                   \
        if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); return 1; } \
    } while (0)

static int cpu_checks() {
    fec::Error err;
    CHECK(!fec::NewRaptorQEncoder({1, 2, 3}, 0, 10, &err) && err.msg == "bad K or L");
    CHECK(!fec::NewRaptorQDecoder(10, 0, &err) && err.msg == "bad dataSize or L");
    auto pk = fec::RaptorQEncodeBlock({1, 2, 3}, 2, 3, 10, &err);
    CHECK(pk.empty() && err.msg == "bad N/K/L");
    auto dec = fec::NewRaptorQDecoder(26 * 16, 16, &err);
    CHECK(dec && !err && dec->K == 26);
    int trues = 0;
    for (uint32_t i = 0; i < 30; ++i) trues += dec->AddSymbol(i, fec::Bytes(16, (uint8_t)i), &err);
    CHECK(trues == 5);  // true from the 26th unique symbol on (RQ/decoder.go:57)
    dec->AddSymbol(40, fec::Bytes(15), &err);
    CHECK(err.code == RQ_ERR_SYMBOL_SIZE && err.msg == "incorrect symbol size 15, should be 16");
    auto d2 = fec::NewRaptorQDecoder(100, 10, &err);
    fec::Bytes out;
    CHECK(!d2->Decode(&out, &err) && err.code == RQ_ERR_NOT_ENOUGH && err.msg == "not enough symbols to decode");
    std::printf("cpu ok\n");
    return 0;
}

static int gpu_checks() {
    std::mt19937_64 rng(1337);
    const int K = 5, L = 1100, N = 8;
    int ok_trials = 0;
    for (int t = 0; t < 50; ++t) {
        fec::Bytes data((size_t)K * L - (t % 7) * 13);
        for (auto& b : data) b = (uint8_t)rng();
        fec::Error err;
        auto pk = fec::RaptorQEncodeBlock(data, N, K, L, &err);
        CHECK(!err && pk.size() == (size_t)N);
        std::vector<fec::Packet> recv;
        for (auto& p : pk)
            if (std::uniform_real_distribution<double>(0, 1)(rng) >= 0.1) recv.push_back(p);
        bool ok = false;
        fec::Bytes got = fec::RaptorQDecodeBytes(recv, N, K, L, (int)data.size(), &ok);
        if (ok) { CHECK(got == data); ++ok_trials; }
        else CHECK(recv.size() < (size_t)K + 1 || got.empty());
    }
    CHECK(ok_trials > 30);
    // GenSymbol of sources aliases the padded payload
    fec::Error err;
    fec::Bytes data(3 * 10 - 4, 7);
    auto enc = fec::NewRaptorQEncoder(data, 3, 10, &err);
    CHECK(enc && enc->BaseSymbolsNum() == 3);
    fec::Bytes s2 = enc->GenSymbol(2);
    CHECK(s2.size() == 10 && s2[5] == 7 && s2[6] == 0 && s2[9] == 0);
    std::printf("gpu ok (%d/50 decoded)\n", ok_trials);
    return 0;
}

int main(int argc, char** argv) {
    const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
    if (cpu_checks()) return 1;
    return gpu ? gpu_checks() : 0;
}
