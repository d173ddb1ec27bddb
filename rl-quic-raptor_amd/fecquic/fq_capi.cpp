// fq_capi.cpp -- C entry points of libfecquic.so for the tests (ctypes): the wire formats, and the
// receiver's non-GPU behaviour mirrored from go/fecquic/rxbuf_test.go:9-100 (ring never blocks,
// ingest stays fast when the ring is full, budget pressure drops repairs only) plus the readiness
// rule (AddSymbol-bool counting, rxbuf.go:472-486).
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "fq_rx.hpp"
#include "fq_wire.hpp"

using namespace fq;

extern "C" {

// fields = {version, scheme, flags, block_id, n, k, sym_id, payload_len, seed_or_idx}
uint32_t fq_header_marshal(const uint32_t fields[9], uint8_t* out) {
    FecHeader h;
    h.version = (uint8_t)fields[0];
    h.scheme = (uint8_t)fields[1];
    h.flags = (uint16_t)fields[2];
    h.block_id = fields[3];
    h.n = fields[4];
    h.k = fields[5];
    h.sym_id = fields[6];
    h.payload_len = fields[7];
    h.seed_or_idx = fields[8];
    return h.version ? marshal(h, out) : marshal_auto(h, out);
}

uint32_t fq_header_unmarshal(const uint8_t* b, uint32_t len, uint32_t fields[9]) {
    FecHeader h;
    const uint32_t n = unmarshal(b, len, &h);
    if (!n) return 0;
    const uint32_t v[9] = {h.version, h.scheme, h.flags, h.block_id, h.n, h.k, h.sym_id, h.payload_len, h.seed_or_idx};
    std::memcpy(fields, v, sizeof v);
    return n;
}

void fq_file_header_marshal(uint64_t size, const uint8_t sha[32], uint32_t chunk_l, uint8_t* out) {
    FileHeader h;
    h.file_size = size;
    std::memcpy(h.sha256, sha, 32);
    h.chunk_l = chunk_l;
    marshal_file(h, out);
}

int fq_file_header_unmarshal(const uint8_t* b, uint32_t len, uint64_t* size, uint8_t sha[32], uint32_t* chunk_l) {
    FileHeader h;
    const int rc = unmarshal_file(b, len, &h);
    if (rc == 0) {
        *size = h.file_size;
        std::memcpy(sha, h.sha256, 32);
        *chunk_l = h.chunk_l;
    }
    return rc;
}

// TestMPSCRingTryPushNonBlocking: fill a ring of `cap`, then `iters` pushes must all fail; returns
// the number that (wrongly) succeeded, and the slowest failed push in ns.
int fq_test_ring(uint32_t cap, uint32_t iters, uint64_t* max_ns) {
    RxManager::Ring r(cap);
    RxManager::Item it;
    for (uint32_t i = 0; i < r.capacity(); ++i) {
        it.esi = i;
        if (!r.try_push(it)) return -1;
    }
    int ok = 0;
    *max_ns = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        ok += r.try_push(it);
        const uint64_t ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                std::chrono::steady_clock::now() - t0).count();
        *max_ns = std::max(*max_ns, ns);
    }
    // drained in order
    std::vector<RxManager::Item> out(r.capacity());
    const uint32_t n = r.try_pop_batch(out.data(), (uint32_t)out.size());
    for (uint32_t i = 0; i < n; ++i)
        if (out[i].esi != i) return -2;
    return n == r.capacity() ? ok : -3;
}

// TestRXIngestNonBlockingWhenRingFull (rxbuf_test.go:37-63): ring of 8, no consumer running; after 8
// ingests, `iters` more must return quickly.  Returns how many took longer than 250 us.
int fq_test_ingest_full(const char* dir, uint32_t iters) {
    RxOptions o;
    o.budget_bytes = 1 << 20;
    o.ring = 8;
    o.decode = false;
    RxManager m(1024, 256, std::string(dir) + "/test.recv", o);
    std::vector<uint8_t> payload(256);
    for (uint32_t i = 0; i < 8; ++i)
        if (!m.ingest(0, i, 8, 4, payload.data(), 256, 256)) return -1;
    int slow = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        (void)m.ingest(0, 1000 + i, 8, 4, payload.data(), 256, 256);
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(250)) ++slow;
    }
    return slow;
}

// TestRXBudgetDropsRepairs (rxbuf_test.go:66-100): budget 3 KiB, K=6 systematic symbols then 2000
// repairs; out = {drops_repairs, drops_system, budget_drop_repairs}.  burst > 0: the repairs come in
// bursts of `burst` with 2 ms pauses, so the ring does not overflow and the classifier's budget rule
// is what drops them -- with K=64 there, so that the block cannot complete during the flood (a
// completed block's late symbols are dropped at ingest instead, fq_test_guards).
int fq_test_budget(const char* dir, uint32_t burst, int64_t out[3]) {
    RxOptions o;
    o.budget_bytes = 3 * 1024;
    o.workers = 1;
    o.ring = 256;
    o.max_n = 4096;  // staging room beyond the budget, as the reference's slab pool is unbounded
    o.max_blocks = 4;
    o.decode = false;
    const uint32_t K = burst ? 64 : 6, N = 2 * K, ds = K * 256;
    RxManager m(burst ? ds : 4096, 256, std::string(dir) + "/budget.recv", o);
    if (m.start() != 0) return -1;
    std::vector<uint8_t> payload(256);
    for (uint32_t i = 0; i < K; ++i)
        if (!m.ingest(0, i, N, K, payload.data(), 256, ds)) return -2;
    for (uint32_t i = 0; i < 2000; ++i) {
        (void)m.ingest(0, K + i, N, K, payload.data(), 256, ds);
        if (burst && i % burst == burst - 1) std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    out[0] = m.stats.drops_repairs.load();
    out[1] = m.stats.drops_system.load();
    out[2] = m.stats.budget_drop_repairs.load();
    uint8_t sha[32] = {};
    (void)m.close_and_finalize(sha, nullptr);
    return 0;
}

// Readiness: one block of K=26, N=32, L=16 with every symbol delivered and no device work.  The
// reference rule (ready at haveU >= K, haveU counting AddSymbol true returns) never readies it, DDL
// or not; the held rule readies it at the 26th symbol.  out = {ready_blocks, queued_by_ddl,
// add_calls, decode_attempts} after `wait_ms`.
int fq_test_ready(const char* dir, int held, int wait_ms, int64_t out[4]) {
    RxOptions o;
    o.decode = false;
    o.ready = held ? RxOptions::READY_HELD : RxOptions::READY_REFERENCE;
    o.ddl_ms = 20;
    RxManager m(26 * 16, 16, std::string(dir) + "/ready.recv", o);
    if (m.start() != 0) return -1;
    std::vector<uint8_t> payload(16);
    for (uint32_t i = 0; i < 32; ++i)
        if (!m.ingest(0, i, 32, 26, payload.data(), 16, 26 * 16)) return -2;
    std::this_thread::sleep_for(std::chrono::milliseconds(wait_ms));
    out[0] = m.stats.ready_blocks.load();
    out[1] = m.stats.queued_by_ddl.load();
    out[2] = m.stats.add_sym_count.load();
    out[3] = m.stats.decode_attempts.load();
    uint8_t sha[32] = {};
    (void)m.close_and_finalize(sha, nullptr);
    return 0;
}

// Ingest guards (network input is untrusted): staging slots are sized from the first header (N=8,
// L=16: 8 rows per slot).  Block 0 (K=4, every source) is decoded on the fast path and written; a
// late repair of it must then be dropped instead of re-creating the block in a fresh slot.  A block
// whose header claims K=40 (more rows than a slot holds), and one with N < K, must be dropped
// without touching the arena.  out = {late symbol accepted, drop_after_q_rep, staging_drops,
// oversized/short header accepted}.
int fq_test_guards(const char* dir, int64_t out[4]) {
    RxOptions o;
    o.decode = false;
    o.ready = RxOptions::READY_HELD;
    o.ddl_ms = 20;
    o.max_blocks = 4;
    RxManager m(64 * 16, 16, std::string(dir) + "/guard.recv", o);
    if (m.start() != 0) return -1;
    std::vector<uint8_t> payload(16, 7);
    for (uint32_t i = 0; i < 4; ++i)
        if (!m.ingest(0, i, 8, 4, payload.data(), 16, 64)) return -2;
    for (int w = 0; w < 100 && m.written() < 64; ++w) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    if (m.written() < 64) return -3;
    out[0] = m.ingest(0, 5, 8, 4, payload.data(), 16, 64) ? 1 : 0;
    out[1] = m.stats.drop_after_q_rep.load();
    const bool big = m.ingest(1, 0, 48, 40, payload.data(), 16, 640);   // K_lib = 40 > 8 rows
    const bool shortn = m.ingest(2, 0, 2, 4, payload.data(), 16, 64);   // N < K
    out[2] = m.stats.staging_drops.load();
    out[3] = (big ? 1 : 0) + (shortn ? 1 : 0);
    uint8_t sha[32] = {};
    (void)m.close_and_finalize(sha, nullptr);
    return 0;
}

}  // extern "C"
