// fq_tx.hpp -- fecquic sender on the GPU engine.
//
// go/fecquic/transfer.go:166-268 reads one K*L block at a time, encodes it with
// fec.RaptorQEncodeBlock (one Solve plus N GenSymbol calls on the CPU, :180) and sends N datagrams
// {16-byte FECHeader}{symbol}.  Here the file is read a window of blocks at a time into pinned
// memory, the window's repair symbols are generated in one rq_encode_batch_host call (GPU), and the
// datagrams are emitted in the reference's order (block by block, ESI 0..N-1) with the same sender
// Bernoulli drop.  The final short block keeps the library's meaning (K = ceil(bytes / L), ESIs from
// there on are repairs, raptorq_wrap.go:81-99) and is encoded on its own.
#pragma once
#include <cstdint>
#include <functional>
#include <string>

namespace fq {

struct TxOptions {
    uint32_t N = 32, K = 26, L = 1200;  // quicfec-client defaults (cmd/quicfec-client/main.go:19-21)
    double drop = 0.0;                  // sender drop probability (transfer.go:203)
    uint64_t seed = 1;
    uint32_t window = 64;               // blocks per GPU encode call
    uint32_t device_mask = 0;
    uint32_t pace_us = 0;               // sleep between windows (the reference paces per datagram)
    int header_version = 0;             // 0: v1 when the block fits it, else v2; 1 or 2: forced
};

struct TxStats {
    uint64_t dgrams = 0, bytes = 0, blocks = 0, dropped = 0, gpu_calls = 0;
    double enc_s = 0, send_s = 0, dur_s = 0;
};

// Emits every datagram of `path` through send(buf, len).  Returns 0, or -1 (I/O), -2 (header does
// not fit the forced version), or an RQ_ERR_* code of the engine.
int send_file(const std::string& path, const TxOptions& o, const std::function<void(const uint8_t*, size_t)>& send,
              TxStats* st);

}  // namespace fq
