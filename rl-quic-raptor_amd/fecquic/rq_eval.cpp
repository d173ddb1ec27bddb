// rq_eval.cpp -- `raptorq_eval` on the GPU engine.
//
// go/cmd/raptorq_eval/main.go with its flags and output lines, for the RaptorQ schemes:
//   -exp B -schemes raptorq,raptorq-batch -N 80 -K 64 -L 1200 -objMB 3 -p 0,0.05,0.1 -trials 10
//          -seed 1337 [-csv out.csv]
//   -exp A -data FILE -K 26 -L 1500 -repeats 200
// Scheme "raptorq" is the reference's loop (main.go:198-228) through the drop-in per-object C-ABI
// (rq_encoder_* / rq_decoder_*, the functions go/fec/raptorq_wrap.go would bind): encode = encoder
// creation, decode = Decode(), and -- unlike the reference, whose GenSymbol calls fall outside both
// timers (main.go:211-219) -- the GenSymbol time is measured too ("gen").  Scheme "raptorq-batch"
// runs the same generations through the batched host-memory API: every full generation of the
// object encoded in one rq_encode_batch_host call and decoded in one rq_decode_batch_host call
// (timers include the PCIe copies); the short final generation goes through the per-object API.
// Loss draws use mt19937_64(seed) instead of Go's math/rand, so patterns differ from the reference's
// for the same seed; rates and timings are comparable.  CSV columns are the reference's
// (main.go:141) plus sum/avg GenSymbol ms.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/rqhip.h"

namespace {

using Clock = std::chrono::steady_clock;
double ms(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

struct Agg {
    int ok = 0, trials = 0;
    double enc = 0, dec = 0, gen = 0;
};

std::string flag(int argc, char** argv, const char* name, const char* def) {
    for (int i = 1; i + 1 < argc; ++i)
        if (std::strcmp(argv[i], name) == 0) return argv[i + 1];
    return def;
}

std::vector<double> parse_p(const std::string& s) {
    std::vector<double> out;
    size_t i = 0;
    while (i < s.size()) {
        size_t j = s.find(',', i);
        if (j == std::string::npos) j = s.size();
        if (j > i) out.push_back(std::atof(s.substr(i, j - i).c_str()));
        i = j + 1;
    }
    return out;
}

// One generation through the per-object API (main.go:198-228).  Returns ok.
bool one_generation(const uint8_t* data, size_t len, int N, int K, int L, double p, std::mt19937_64& rng, Agg& a,
                    std::vector<uint8_t>& out) {
    (void)K;
    std::uniform_real_distribution<double> u(0, 1);
    int err = 0;
    auto t0 = Clock::now();
    rq_enc* enc = rq_encoder_create(data, len, (uint32_t)L, &err);
    if (!enc) return false;
    a.enc += ms(t0, Clock::now());
    rq_dec* dec = rq_decoder_create(len, (uint32_t)L, &err);
    if (!dec) { rq_encoder_free(enc); return false; }
    std::vector<uint8_t> sym(L);
    bool ok = true;
    for (int i = 0; i < N; ++i) {
        if (u(rng) < p) continue;
        auto tg = Clock::now();
        if (rq_encoder_symbol(enc, (uint32_t)i, sym.data()) != RQ_OK) { ok = false; break; }
        a.gen += ms(tg, Clock::now());
        int can = 0;
        if (rq_decoder_add(dec, (uint32_t)i, sym.data(), sym.size(), &can) != RQ_OK) { ok = false; break; }
    }
    out.assign(len, 0);
    int dok = 0;
    auto t1 = Clock::now();
    const int rc = ok ? rq_decoder_decode(dec, out.data(), &dok) : -1;
    a.dec += ms(t1, Clock::now());
    rq_decoder_free(dec);
    rq_encoder_free(enc);
    return ok && rc == RQ_OK && dok && std::memcmp(out.data(), data, len) == 0;
}

// All full generations of the object in one batched call each way; the short tail per object.
bool batch_trial(const std::vector<uint8_t>& obj, int N, int K, int L, double p, std::mt19937_64& rng, Agg& a) {
    std::uniform_real_distribution<double> u(0, 1);
    const size_t blk = (size_t)K * L;
    const uint32_t nb = (uint32_t)(obj.size() / blk), R = (uint32_t)(N - K);
    bool ok = true;
    if (nb) {
        std::vector<uint32_t> esi(R);
        for (uint32_t i = 0; i < R; ++i) esi[i] = K + i;
        uint8_t* rep = static_cast<uint8_t*>(rq_host_alloc((size_t)nb * R * L + 1));
        uint8_t* data = static_cast<uint8_t*>(rq_host_alloc(nb * blk));
        auto t0 = Clock::now();
        rq_encode_desc e{};
        e.T = L; e.K = K; e.n_blocks = nb; e.src = obj.data(); e.src_stride = blk;
        e.n_esi = R; e.esi = esi.data(); e.out = rep; e.out_stride = (uint64_t)R * L;
        if (rq_encode_batch_host(&e, 0) != RQ_OK) ok = false;
        a.enc += ms(t0, Clock::now());
        std::vector<uint32_t> ne(nb), nr(nb), er, re;
        std::vector<uint8_t> rows;
        std::memcpy(data, obj.data(), nb * blk);
        for (uint32_t b = 0; b < nb; ++b) {
            for (int i = 0; i < N; ++i) {
                const bool lost = u(rng) < p;
                if (i < K && lost) { er.push_back(i); ne[b]++; std::memset(data + b * blk + (size_t)i * L, 0, L); }
                if (i >= K && !lost) {
                    re.push_back(i);
                    nr[b]++;
                    rows.insert(rows.end(), rep + ((size_t)b * R + (i - K)) * L, rep + ((size_t)b * R + (i - K) + 1) * L);
                }
            }
        }
        er.push_back(0);
        re.push_back(0);
        std::vector<int32_t> st(nb);
        rq_decode_desc d{};
        d.T = L; d.K = K; d.n_blocks = nb; d.data = data; d.data_stride = blk; d.n_erased = ne.data();
        d.erased = er.data(); d.n_repair = nr.data(); d.repair_esi = re.data(); d.repair = rows.data();
        d.status = st.data();
        auto t1 = Clock::now();
        if (rq_decode_batch_host(&d, 0) != RQ_OK) ok = false;
        a.dec += ms(t1, Clock::now());
        for (uint32_t b = 0; b < nb && ok; ++b)
            ok = st[b] == 1 && std::memcmp(data + b * blk, obj.data() + b * blk, blk) == 0;
        rq_host_free(rep);
        rq_host_free(data);
    }
    const size_t tail = obj.size() - (size_t)nb * blk;
    if (tail && ok) {
        std::vector<uint8_t> out;
        ok = one_generation(obj.data() + (size_t)nb * blk, tail, N, K, L, p, rng, a, out);
    }
    return ok;
}

int exp_b(int argc, char** argv) {
    const int N = std::atoi(flag(argc, argv, "-N", "32").c_str()), K = std::atoi(flag(argc, argv, "-K", "26").c_str());
    const int L = std::atoi(flag(argc, argv, "-L", "1500").c_str());
    const int objMB = std::atoi(flag(argc, argv, "-objMB", "3").c_str());
    const int trials = std::atoi(flag(argc, argv, "-trials", "10").c_str());
    const uint64_t seed = std::strtoull(flag(argc, argv, "-seed", "1337").c_str(), nullptr, 10);
    const std::vector<double> ps = parse_p(flag(argc, argv, "-p", "0,0.001,0.005,0.01,0.05,0.10,0.15"));
    const std::string schemes = flag(argc, argv, "-schemes", "raptorq");
    const std::string csv = flag(argc, argv, "-csv", "");
    if (K <= 0 || N < K || L <= 0) { std::printf("bad N/K/L\n"); return 1; }
    std::vector<uint8_t> obj((size_t)objMB << 20);
    std::mt19937_64 fill(seed ^ 0x9E3779B97F4A7C15ull);
    for (auto& b : obj) b = (uint8_t)fill();
    std::mt19937_64 rng(seed);
    FILE* cf = nullptr;
    if (!csv.empty()) {
        cf = std::fopen(csv.c_str(), "a");
        if (cf && std::ftell(cf) == 0)
            std::fprintf(cf, "scheme,p,trials,ok_rate,sum_encode_ms,avg_encode_ms,sum_decode_ms,avg_decode_ms,N,K,L,seed,"
                             "sum_gensymbol_ms,avg_gensymbol_ms\n");
    }
    size_t i0 = 0;
    while (i0 < schemes.size()) {
        size_t j = schemes.find(',', i0);
        if (j == std::string::npos) j = schemes.size();
        const std::string scheme = schemes.substr(i0, j - i0);
        i0 = j + 1;
        if (scheme != "raptorq" && scheme != "raptorq-batch") continue;  // other codes stay in the reference
        for (double p : ps) {
            Agg a;
            a.trials = trials;
            for (int t = 0; t < trials; ++t) {
                bool ok = true;
                if (scheme == "raptorq") {
                    std::vector<uint8_t> out;
                    for (size_t off = 0; off < obj.size();) {
                        const size_t end = std::min(obj.size(), off + (size_t)K * L);
                        ok &= one_generation(obj.data() + off, end - off, N, K, L, p, rng, a, out);
                        off = end;
                    }
                } else {
                    ok = batch_trial(obj, N, K, L, p, rng, a);
                }
                a.ok += ok;
            }
            const double rate = (double)a.ok / a.trials;
            std::printf("scheme=%s p=%.4f ok=%.4f enc(total)=%.1fms dec(total)=%.1fms gen(total)=%.1fms\n",
                        scheme.c_str(), p, rate, a.enc, a.dec, a.gen);
            if (cf)
                std::fprintf(cf, "%s,%.6f,%d,%.6f,%.3f,%.6f,%.3f,%.6f,%d,%d,%d,%llu,%.3f,%.6f\n", scheme.c_str(), p,
                             trials, rate, a.enc, a.enc / trials, a.dec, a.dec / trials, N, K, L,
                             (unsigned long long)seed, a.gen, a.gen / trials);
        }
    }
    if (cf) std::fclose(cf);
    return 0;
}

int exp_a(int argc, char** argv) {  // main.go:65-117
    const std::string path = flag(argc, argv, "-data", "test_data/train_FD001.txt");
    const int K = std::atoi(flag(argc, argv, "-K", "26").c_str()), L = std::atoi(flag(argc, argv, "-L", "1500").c_str());
    const int repeats = std::atoi(flag(argc, argv, "-repeats", "200").c_str());
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { std::printf("read %s: no such file\n", path.c_str()); return 1; }
    std::vector<uint8_t> src;
    uint8_t buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) src.insert(src.end(), buf, buf + n);
    std::fclose(f);
    double enc = 0, dec = 0;
    std::vector<uint8_t> sym(L), out;
    for (int r = 0; r < repeats; ++r) {
        for (size_t off = 0; off < src.size();) {
            const size_t end = std::min(src.size(), off + (size_t)K * L);
            int err = 0;
            auto t0 = Clock::now();
            rq_enc* e = rq_encoder_create(src.data() + off, end - off, L, &err);
            if (!e) { std::printf("encoder: %s\n", rq_last_error()); return 1; }
            enc += ms(t0, Clock::now());
            rq_dec* d = rq_decoder_create(end - off, L, &err);
            for (int i = 0; i < K; ++i) {
                rq_encoder_symbol(e, i, sym.data());
                int can;
                rq_decoder_add(d, i, sym.data(), sym.size(), &can);
            }
            out.assign(end - off, 0);
            int ok = 0;
            auto t1 = Clock::now();
            if (rq_decoder_decode(d, out.data(), &ok) != RQ_OK || !ok) { std::printf("decode fail\n"); return 1; }
            dec += ms(t1, Clock::now());
            if (std::memcmp(out.data(), src.data() + off, out.size()) != 0) { std::printf("mismatch at rep %d\n", r); return 1; }
            rq_decoder_free(d);
            rq_encoder_free(e);
            off = end;
        }
    }
    std::printf("Experiment A: RaptorQ p=0 enc(total)=%.3fms dec(total)=%.3fms (repeats=%d)\n", enc, dec, repeats);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    const std::string exp = flag(argc, argv, "-exp", "A");
    if (exp == "A" || exp == "a") return exp_a(argc, argv);
    if (exp == "B" || exp == "b") return exp_b(argc, argv);
    std::printf("unknown exp; use A or B\n");
    return 0;
}
