// fq_rx.cpp -- fecquic receiver on the GPU engine (see fq_rx.hpp).
#include "fq_rx.hpp"

#include <fcntl.h>
#include <openssl/evp.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "../../include/rqhip.h"

namespace fq {

// ---------------------------------------------------------------- ring
RxManager::Ring::Ring(uint32_t cap) : slots(std::max<uint32_t>(2, [&] {
                                          uint32_t n = 1;
                                          while (n < cap) n <<= 1;
                                          return n;
                                      }())) {
    mask = slots.size() - 1;
    for (size_t i = 0; i < slots.size(); ++i) slots[i].seq.store(i, std::memory_order_relaxed);
}

bool RxManager::Ring::try_push(const Item& x) {
    uint64_t pos = tail.load(std::memory_order_relaxed);
    for (;;) {
        Slot& s = slots[pos & mask];
        const uint64_t seq = s.seq.load(std::memory_order_acquire);
        const int64_t dif = (int64_t)seq - (int64_t)pos;
        if (dif == 0) {
            if (tail.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
                s.v = x;
                s.seq.store(pos + 1, std::memory_order_release);
                return true;
            }
        } else if (dif < 0) {
            return false;  // full: the slot still holds an item the consumer has not taken
        } else {
            pos = tail.load(std::memory_order_relaxed);
        }
    }
}

uint32_t RxManager::Ring::try_pop_batch(Item* dst, uint32_t max) {
    uint32_t n = 0;
    while (n < max) {
        Slot& s = slots[head & mask];
        const uint64_t seq = s.seq.load(std::memory_order_acquire);
        if ((int64_t)seq - (int64_t)(head + 1) < 0) break;  // not yet published
        dst[n++] = s.v;
        s.seq.store(head + mask + 1, std::memory_order_release);
        ++head;
    }
    return n;
}

// ---------------------------------------------------------------- sha-256
void sha256_buf(const uint8_t* p, size_t n, uint8_t out[32]) {
    unsigned int len = 32;
    EVP_Digest(p, n, out, &len, EVP_sha256(), nullptr);
}

bool sha256_file(const std::string& path, uint8_t out[32]) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return false;
    EVP_MD_CTX* c = EVP_MD_CTX_new();
    EVP_DigestInit_ex(c, EVP_sha256(), nullptr);
    std::vector<uint8_t> buf(1 << 20);
    ssize_t r;
    while ((r = ::read(fd, buf.data(), buf.size())) > 0) EVP_DigestUpdate(c, buf.data(), (size_t)r);
    unsigned int len = 32;
    EVP_DigestFinal_ex(c, out, &len);
    EVP_MD_CTX_free(c);
    ::close(fd);
    return r == 0;
}

// ---------------------------------------------------------------- manager
RxManager::RxManager(uint64_t file_size, uint32_t L, std::string out_path, RxOptions o)
    : file_size_(file_size), L_(L), out_path_(std::move(out_path)), o_(o), ring_(o.ring) {
    tmp_path_ = out_path_ + ".part";
}

RxManager::~RxManager() {
    if (started_ && !stop_.load()) {
        stop_ = true;
        qcv_.notify_all();
        wcv_.notify_all();
        for (auto& t : threads_) t.join();
    }
    for (auto& kv : blocks_) delete kv.second;
    for (Block* b : decode_q_) (void)b;
    if (arena_) {
        if (arena_pinned_) rq_host_free(arena_);
        else std::free(arena_);
    }
    if (fd_ >= 0) ::close(fd_);
}

int RxManager::start() {
    fd_ = ::open(tmp_path_.c_str(), O_CREAT | O_TRUNC | O_RDWR, 0644);
    if (fd_ < 0) { err_ = "cannot create " + tmp_path_; return -2; }
    if (::ftruncate(fd_, (off_t)file_size_) != 0) { err_ = "truncate failed"; return -2; }
    started_ = true;
    threads_.emplace_back(&RxManager::classifier, this);
    threads_.emplace_back(&RxManager::ddl_ticker, this);
    for (int i = 0; i < std::max(1, o_.workers); ++i) threads_.emplace_back(&RxManager::decoder, this);
    threads_.emplace_back(&RxManager::writer, this);
    return 0;
}

bool RxManager::ingest(uint32_t block_id, uint32_t esi, uint32_t N, uint32_t K, const uint8_t* data, uint32_t len,
                       uint32_t data_size) {
    const bool repair_wire = esi >= K;  // rxbuf.go:499 (wire K)
    Item it;
    it.block_id = block_id;
    it.esi = esi;
    it.len = len;
    it.repair = repair_wire;
    it.row = UINT32_MAX;  // not staged
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (!arena_) {  // staging is sized from the first header: max_n symbols of L bytes per block
            const uint32_t mn = o_.max_n ? o_.max_n : N;
            slot_bytes_ = (size_t)std::max(mn, K) * L_;
            const size_t bytes = slot_bytes_ * o_.max_blocks;
            arena_ = o_.decode ? static_cast<uint8_t*>(rq_host_alloc(bytes)) : nullptr;
            arena_pinned_ = arena_ != nullptr;
            if (!arena_) arena_ = static_cast<uint8_t*>(std::malloc(bytes));
            for (uint32_t s = o_.max_blocks; s-- > 0;) free_slots_.push_back(s);
        }
        auto f = blocks_.find(block_id);
        Block* b = f == blocks_.end() ? nullptr : f->second;
        if (!b && finished_.count(block_id)) {
            // a late or reordered symbol of a block already written: the reference re-creates the block
            // (rxbuf.go:437); here that would pin a staging slot that never decodes, so it is dropped
            if (repair_wire) { stats.drop_after_q_rep++; stats.drops_repairs++; }
            else { stats.drop_after_q_sys++; stats.drops_system++; }
            return false;
        }
        if (!b) {
            // the header's own sizes must fit the block's staging slot (sized from the first header):
            // the library K = ceil(data_size / L) source rows, and N >= K on the wire
            const uint64_t k_lib = data_size ? ((uint64_t)data_size + L_ - 1) / L_ : 0;
            if (free_slots_.empty() || len != L_ || data_size == 0 || N < K ||
                std::max<uint64_t>(N, k_lib) * L_ > slot_bytes_) {
                stats.staging_drops++;
                if (repair_wire) stats.drops_repairs++;
                else stats.drops_system++;
                return false;
            }
            b = new Block();
            b->id = block_id;
            b->k_wire = K;
            b->n = N;
            b->data_size = data_size;
            b->K = (data_size + L_ - 1) / L_;  // library K (RQ/params.go:36): the decoder's own K
            b->slot = free_slots_.back();
            free_slots_.pop_back();
            b->t0 = Clock::now();
            b->data = arena_ + (size_t)b->slot * slot_bytes_;
            b->rep = b->data + (size_t)b->K * L_;
            b->rep_cap = (uint32_t)((slot_bytes_ - (size_t)b->K * L_) / L_);
            b->have.assign(b->K, 0);
            blocks_[block_id] = b;
        }
        // staging a symbol while a decode attempt reads the block is safe only for repairs (appended
        // past the rows the attempt uses); the reference drops every symbol of a queued block
        // (rxbuf.go:445-458), which READY_HELD relaxes for repairs so that a rank-deficient attempt
        // at exactly K symbols can be retried with the ones that arrived meanwhile
        const bool stage = !b->done && len == L_ &&
                           (!b->queued || (o_.ready == RxOptions::READY_HELD && esi >= b->K));
        if (stage) {
            if (esi < b->K) {
                std::memcpy(b->data + (size_t)esi * L_, data, L_);
                it.row = esi;
            } else if (b->rep_rows < b->rep_cap) {
                it.row = b->rep_rows++;
                std::memcpy(b->rep + (size_t)it.row * L_, data, L_);
            } else {
                stats.staging_drops++;
                stats.drops_repairs++;
                return false;
            }
            it.gen = b->gen;
        }
    }
    if (!ring_.try_push(it)) {
        if (repair_wire) { stats.drops_repairs++; stats.ring_drop_repairs++; }
        else { stats.drops_system++; stats.ring_drop_system++; }
        return false;
    }
    return true;
}

void RxManager::classifier() {  // rxbuf.go:406-493
    std::vector<Item> buf(64);
    while (!stop_.load()) {
        const uint32_t n = ring_.try_pop_batch(buf.data(), (uint32_t)buf.size());
        if (n == 0) {
            std::this_thread::sleep_for(std::chrono::microseconds(200));
            continue;
        }
        for (uint32_t i = 0; i < n; ++i) {
            const Item& s = buf[i];
            if (in_use_.load() + s.len > (int64_t)o_.budget_bytes && s.repair) {  // :425-431
                stats.drops_repairs++;
                stats.budget_drop_repairs++;
                continue;
            }
            std::unique_lock<std::mutex> lk(mu_);
            auto f = blocks_.find(s.block_id);
            if (f == blocks_.end()) continue;
            Block* b = f->second;
            const bool late_ok = o_.ready == RxOptions::READY_HELD && s.esi >= b->K;
            if ((b->queued && !late_ok) || b->done || s.row == UINT32_MAX || s.gen != b->gen) {  // :445-458
                if (s.repair) stats.drop_after_q_rep++;
                else { stats.drop_after_q_sys++; stats.drops_system++; }
                continue;
            }
            bool dup;
            if (s.esi < b->K) {
                dup = b->have[s.esi] != 0;
                if (!dup) { b->have[s.esi] = 1; b->nsrc++; }
            } else {
                dup = !b->seen.insert(s.esi).second;
                if (!dup) { b->acc_rows.push_back(s.row); b->acc_esi.push_back(s.esi); }
            }
            if (dup) {  // :459-466
                stats.dup_symbols++;
                continue;
            }
            in_use_ += s.len;
            b->bytes += s.len;
            stats.add_sym_count++;
            // AddSymbol's bool: K <= unique symbols held (RQ/decoder.go:47,57)
            const bool inc = b->K <= b->nsrc + (uint32_t)b->acc_esi.size();
            bool ready = false;
            if (o_.ready == RxOptions::READY_REFERENCE) {
                if (inc && ++b->have_u >= b->k_wire && !b->queued) ready = true;  // :476-486
            } else if (inc && !b->queued) {
                ready = true;
            }
            if (ready) {
                stats.ready_blocks++;
                stats.ready_us += std::chrono::duration_cast<std::chrono::microseconds>(Clock::now() - b->t0).count();
                stats.queued_by_ready++;
                b->queued = true;
                lk.unlock();
                std::lock_guard<std::mutex> q(qmu_);
                decode_q_.push_back(b);
                qcv_.notify_one();
            }
        }
    }
}

void RxManager::ddl_ticker() {  // rxbuf.go:379-404
    while (!stop_.load()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
        const auto now = Clock::now();
        std::vector<Block*> due;
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (auto& kv : blocks_) {
                Block* b = kv.second;
                if (b->done || b->queued) continue;
                if (now - b->t0 >= std::chrono::milliseconds(o_.ddl_ms)) {
                    b->queued = true;
                    stats.queued_by_ddl++;
                    due.push_back(b);
                }
            }
        }
        if (!due.empty()) {
            std::lock_guard<std::mutex> q(qmu_);
            for (Block* b : due) decode_q_.push_back(b);
            qcv_.notify_all();
        }
    }
}

void RxManager::decoder() {  // rxbuf.go:336-377, one GPU call per batch of ready blocks
    while (true) {
        std::vector<Block*> got;
        {
            std::unique_lock<std::mutex> q(qmu_);
            qcv_.wait(q, [&] { return stop_.load() || !decode_q_.empty(); });
            if (stop_.load()) return;
            while (!decode_q_.empty() && got.size() < o_.batch) {
                got.push_back(decode_q_.front());
                decode_q_.pop_front();
            }
        }
        // snapshot under the lock: which blocks to decode, their erased rows and received repairs
        struct Job {
            Block* b;
            std::vector<uint32_t> erased, rep_esi;  // snapshot: the classifier may append meanwhile
        };
        std::map<uint32_t, std::vector<Job>> by_k;  // one rq_decode_blocks_host call per K
        std::vector<Block*> ok_now;
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (Block* b : got) {
                if (b->done) continue;
                const uint32_t held = b->nsrc + (uint32_t)b->acc_esi.size();
                if ((o_.ready == RxOptions::READY_REFERENCE && b->have_u < b->k_wire) || held < b->K) {
                    b->queued = false;  // not ready yet (:344-348)
                    continue;
                }
                stats.decode_attempts++;
                Job j{b, {}};
                for (uint32_t i = 0; i < b->K; ++i)
                    if (!b->have[i]) j.erased.push_back(i);
                if (j.erased.empty()) {  // all K sources held: the library's fast path, no solve
                    stats.fast_path_blocks++;
                    ok_now.push_back(b);
                    continue;
                }
                // received repair rows consecutive in acceptance order (ascending rows: compaction
                // moves each down over the rows of dropped or duplicate symbols)
                for (size_t r = 0; r < b->acc_rows.size(); ++r)
                    if (b->acc_rows[r] != r) {
                        std::memmove(b->rep + r * L_, b->rep + (size_t)b->acc_rows[r] * L_, L_);
                        b->acc_rows[r] = (uint32_t)r;
                    }
                b->rep_rows = (uint32_t)b->acc_rows.size();
                ++b->gen;  // rows staged but not yet classified may have been moved: drop them
                j.rep_esi = b->acc_esi;
                by_k[b->K].push_back(std::move(j));
            }
        }
        std::vector<std::pair<Block*, bool>> results;
        for (Block* b : ok_now) results.push_back({b, true});
        for (auto& kv : by_k) {
            std::vector<rq_block_io> io(kv.second.size());
            for (size_t i = 0; i < io.size(); ++i) {
                Block* b = kv.second[i].b;
                io[i].data = b->data;
                io[i].repair = b->rep;
                io[i].n_erased = (uint32_t)kv.second[i].erased.size();
                io[i].erased = kv.second[i].erased.data();
                io[i].n_repair = (uint32_t)kv.second[i].rep_esi.size();
                io[i].repair_esi = kv.second[i].rep_esi.data();
                io[i].status = 0;
            }
            const auto t0 = Clock::now();
            int rc = o_.decode ? rq_decode_blocks_host(kv.first, L_, io.data(), (uint32_t)io.size(), o_.device_mask)
                               : RQ_ERR_DEVICE;
            stats.gpu_calls++;
            stats.dec_us += std::chrono::duration_cast<std::chrono::microseconds>(Clock::now() - t0).count();
            if (rc != RQ_OK) {
                std::lock_guard<std::mutex> lk(mu_);
                err_ = rq_last_error();
            }
            for (size_t i = 0; i < io.size(); ++i) results.push_back({kv.second[i].b, rc == RQ_OK && io[i].status == 1});
        }
        std::vector<Block*> to_write;
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (auto& r : results) {
                if (r.second) {
                    r.first->done = true;
                    stats.dec_blocks++;
                    to_write.push_back(r.first);
                } else {  // decoding failed; likely need more symbols (:352-357)
                    stats.decode_failures++;
                    r.first->queued = false;
                }
            }
        }
        if (!to_write.empty()) {
            std::lock_guard<std::mutex> w(wmu_);
            for (Block* b : to_write) write_q_.push_back(b);
            wcv_.notify_one();
        }
    }
}

void RxManager::writer() {  // rxbuf.go:317-334
    while (true) {
        Block* b;
        {
            std::unique_lock<std::mutex> w(wmu_);
            wcv_.wait(w, [&] { return stop_.load() || !write_q_.empty(); });
            if (write_q_.empty()) return;
            b = write_q_.front();
            write_q_.pop_front();
        }
        const uint64_t off = (uint64_t)b->id * b->k_wire * L_;  // rxbuf.go:360
        uint64_t n = b->data_size;
        if (off >= file_size_) n = 0;
        else n = std::min<uint64_t>(n, file_size_ - off);
        const auto t0 = Clock::now();
        uint64_t done = 0;
        while (done < n) {
            const ssize_t r = ::pwrite(fd_, b->data + done, n - done, (off_t)(off + done));
            if (r <= 0) break;
            done += (uint64_t)r;
        }
        stats.write_us += std::chrono::duration_cast<std::chrono::microseconds>(Clock::now() - t0).count();
        written_ += done;
        release(b);
    }
}

void RxManager::release(Block* b) {
    std::lock_guard<std::mutex> lk(mu_);
    in_use_ -= (int64_t)b->bytes;
    auto f = blocks_.find(b->id);
    if (f != blocks_.end() && f->second == b) blocks_.erase(f);
    finished_.insert(b->id);
    free_slots_.push_back(b->slot);
    delete b;
}

int RxManager::close_and_finalize(const uint8_t sha[32], std::string* final_path) {
    stop_ = true;
    qcv_.notify_all();
    wcv_.notify_all();
    for (auto& t : threads_) t.join();
    threads_.clear();
    if (fd_ >= 0) { ::close(fd_); fd_ = -1; }
    uint8_t got[32];
    if (!sha256_file(tmp_path_, got)) return -2;
    if (std::memcmp(got, sha, 32) != 0) return -1;  // "sha256 mismatch" (rxbuf.go:560-562)
    if (std::rename(tmp_path_.c_str(), out_path_.c_str()) != 0) return -2;
    if (final_path) *final_path = out_path_;
    return 0;
}

}  // namespace fq
