// fq_rx.hpp -- fecquic receiver on the GPU engine.
//
// Mirrors go/fecquic/rxbuf.go: an ingest call per datagram (non-blocking; a bounded MPSC ring into a
// single classifier thread), a classifier that applies the budget (repairs only), de-duplication and
// the decoder's AddSymbol bool, a 50 ms decode deadline (DDL) ticker, decode workers and an offset
// writer with a SHA-256 check at the end.  What changes, MI355X-first:
//   * ingest copies each payload straight into the block's staging area in pinned host memory (source
//     row i at data + i*L, repairs appended), which is what the GPU decode uploads from -- the one
//     host copy the reference also makes (its slab copy, rxbuf.go:497-507), and no second copy into a
//     decoder object (the reference's AddSymbol copy, RQ/decoder.go:39-57);
//   * decode workers take every ready block at once and decode them in one rq_decode_blocks_host call
//     (GPU syndrome decode), instead of one Decode() per block (rxbuf.go:336-377).
// The AddSymbol bool is kept bit for bit (true once K <= unique symbols held, RQ/decoder.go:47,57),
// and so is the reference's readiness rule (haveU counts true returns, ready at haveU >= K,
// rxbuf.go:472-486, :344-348) -- see Ready.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

namespace fq {

using Clock = std::chrono::steady_clock;

struct RxOptions {
    uint64_t budget_bytes = 10ull << 20;  // rxbuf.go:24-26
    int ddl_ms = 50;                      // rxbuf.go:27-29
    int workers = 1;                      // decode workers (each drives whole batches on the GPU)
    uint32_t ring = 4096;                 // ingress ring slots (rounded up to a power of two)
    uint32_t max_blocks = 256;            // blocks in flight (pinned staging slots)
    uint32_t max_n = 0;                   // symbols staged per block (0: N of the first header)
    uint32_t batch = 256;                 // blocks per GPU decode call
    uint32_t device_mask = 0;
    // READY_REFERENCE: rxbuf.go's rule -- haveU counts AddSymbol true returns and a block is decoded
    // once haveU >= K (so it needs 2K-1 unique symbols; with N < 2K-1 a block never decodes, DDL or
    // not, because the worker skips blocks with haveU < K, rxbuf.go:344-348).  READY_HELD: decode as
    // soon as the first true is returned (K unique symbols held), the evident intent.
    enum Ready { READY_REFERENCE = 0, READY_HELD = 1 } ready = READY_REFERENCE;
    bool decode = true;  // false: no device work (classifier tests)
};

struct RxStats {
    std::atomic<int64_t> dec_blocks{0}, dec_us{0}, drops_repairs{0}, drops_system{0}, ring_drop_repairs{0},
        ring_drop_system{0}, budget_drop_repairs{0}, dup_symbols{0}, drop_after_q_rep{0}, drop_after_q_sys{0},
        add_sym_count{0}, decode_attempts{0}, decode_failures{0}, queued_by_ddl{0}, queued_by_ready{0},
        ready_blocks{0}, ready_us{0}, gpu_calls{0}, fast_path_blocks{0}, write_us{0}, staging_drops{0};
};

class RxManager {
public:
    // out_path: the final file; data is written to out_path + ".part" and renamed after the SHA-256
    // check (rxbuf.go:297-312, 540-566).
    RxManager(uint64_t file_size, uint32_t L, std::string out_path, RxOptions o);
    ~RxManager();
    int start();  // 0 ok
    // One received symbol (rxbuf.go:497-538): false if dropped at ingress (ring full, no staging).
    bool ingest(uint32_t block_id, uint32_t esi, uint32_t N, uint32_t K, const uint8_t* data, uint32_t len,
                uint32_t data_size);
    // Stops the pipeline, verifies the SHA-256 and renames the file: 0 ok, -1 mismatch, -2 I/O.
    int close_and_finalize(const uint8_t sha[32], std::string* final_path);
    uint64_t written() const { return written_.load(); }
    uint64_t in_use() const { return (uint64_t)in_use_.load(); }
    bool ring_full() const { return ring_.full(); }
    RxStats stats;
    const std::string& last_error() const { return err_; }

    // exposed for tests
    struct Item {
        uint32_t block_id = 0, esi = 0, row = 0, len = 0, gen = 0;
        bool repair = false;
    };
    struct Ring {  // bounded MPSC ring with per-slot sequence numbers (non-blocking push/pop)
        explicit Ring(uint32_t cap);
        bool try_push(const Item& x);
        uint32_t try_pop_batch(Item* dst, uint32_t max);
        uint32_t capacity() const { return (uint32_t)slots.size(); }
        bool full() const {  // the next push would fail (its slot still holds an unconsumed item)
            const uint64_t pos = tail.load(std::memory_order_relaxed);
            return (int64_t)slots[pos & mask].seq.load(std::memory_order_acquire) - (int64_t)pos < 0;
        }
        struct Slot {
            std::atomic<uint64_t> seq;
            Item v;
        };
        std::vector<Slot> slots;
        uint64_t mask;
        std::atomic<uint64_t> tail{0};
        uint64_t head = 0;
    };

private:
    struct Block {
        uint32_t id = 0, k_wire = 0, n = 0, data_size = 0, K = 0, slot = 0;
        Clock::time_point t0;
        uint8_t* data = nullptr;  // K*L, pinned
        uint8_t* rep = nullptr;   // rep_cap rows of L, pinned
        uint32_t rep_cap = 0, rep_rows = 0;
        std::vector<uint8_t> have;
        uint32_t nsrc = 0, have_u = 0;
        std::vector<uint32_t> acc_rows, acc_esi;
        std::unordered_set<uint32_t> seen;
        bool queued = false, done = false;
        uint32_t gen = 0;    // staging generation: bumped when a decode attempt compacts the rows
        uint64_t bytes = 0;  // accepted bytes (budget accounting)
    };
    void classifier();
    void ddl_ticker();
    void decoder();
    void writer();
    void release(Block* b);

    uint64_t file_size_;
    uint32_t L_;
    std::string out_path_, tmp_path_, err_;
    RxOptions o_;
    int fd_ = -1;
    uint8_t* arena_ = nullptr;
    bool arena_pinned_ = false;
    size_t slot_bytes_ = 0;
    std::vector<uint32_t> free_slots_;
    std::mutex mu_;
    std::map<uint32_t, Block*> blocks_;
    std::unordered_set<uint32_t> finished_;  // ids of blocks already written (their late symbols drop)
    Ring ring_;
    std::atomic<int64_t> in_use_{0};
    std::atomic<uint64_t> written_{0};
    std::atomic<bool> stop_{false};
    std::mutex qmu_;
    std::condition_variable qcv_;
    std::deque<Block*> decode_q_;
    std::mutex wmu_;
    std::condition_variable wcv_;
    std::deque<Block*> write_q_;
    std::vector<std::thread> threads_;
    bool started_ = false;
};

// SHA-256 of a file's first `size` bytes (the fecquic file header digest, fileheader.go:59-80).
bool sha256_file(const std::string& path, uint8_t out[32]);
void sha256_buf(const uint8_t* p, size_t n, uint8_t out[32]);

}  // namespace fq
