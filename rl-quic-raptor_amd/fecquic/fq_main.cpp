// fq_main.cpp -- `fecquic`: a loopback file transfer through the GPU engine in the shape of
// go/fecquic (client: transfer.go:42-282, server: transfer.go:291-479), for SURVEY.md sec. 8(f).
//
//   fecquic loopback --file F --out PATH [--K 26 --N 32 --L 1200 --drop 0 --seed 1 --window 64
//                    --transport inproc|udp --ready ref|held --workers 1 --ddl-ms 50 --budget BYTES
//                    --max-blocks 128 --ring 4096 --header-version 0|1|2 --timeout-s 120 --dump PATH]
//
// The file header ("QFEC", size, SHA-256, L) travels first on a reliable channel (a TCP connection
// for --transport udp, standing in for the QUIC stream of transfer.go:94-114), then every symbol as
// one datagram {FECHeader}{L bytes} (UDP on 127.0.0.1, or handed straight to the receiver's ingest
// for --transport inproc).  The receiver decodes on the GPU, writes at id*K*L, checks the SHA-256 and
// renames the file.  Prints one JSON line with the outcome and the sender/receiver counters.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rqhip.h"
#include "fq_rx.hpp"
#include "fq_tx.hpp"
#include "fq_wire.hpp"

using namespace fq;

namespace {

// Receiver side of one datagram (transfer.go:382-411): header, scheme check, then ingest with the
// block's exact byte count remAtPos.
void deliver(RxManager& rx, const FileHeader& fh, const uint8_t* b, size_t n) {
    FecHeader h;
    const uint32_t hl = unmarshal(b, (uint32_t)n, &h);
    if (!hl || h.scheme != SCHEME_RAPTORQ) return;
    if (h.payload_len > n - hl) return;
    const uint64_t max_block = (uint64_t)h.k * fh.chunk_l;
    const uint64_t before = (uint64_t)h.block_id * max_block;
    if (before >= fh.file_size) return;
    const uint64_t rem = std::min<uint64_t>(fh.file_size - before, max_block);
    rx.ingest(h.block_id, h.sym_id, h.n, h.k, b + hl, h.payload_len, (uint32_t)rem);
}

std::string arg(int argc, char** argv, const char* name, const char* def) {
    for (int i = 2; i + 1 < argc; ++i)
        if (std::strcmp(argv[i], name) == 0) return argv[i + 1];
    return def;
}

void hex(const uint8_t* p, char* out) {
    for (int i = 0; i < 32; ++i) std::snprintf(out + 2 * i, 3, "%02x", p[i]);
}

int loopback(int argc, char** argv) {
    const std::string file = arg(argc, argv, "--file", ""), out = arg(argc, argv, "--out", "");
    if (file.empty() || out.empty()) { std::fprintf(stderr, "need --file and --out\n"); return 2; }
    TxOptions to;
    to.K = (uint32_t)std::atoi(arg(argc, argv, "--K", "26").c_str());
    to.N = (uint32_t)std::atoi(arg(argc, argv, "--N", "32").c_str());
    to.L = (uint32_t)std::atoi(arg(argc, argv, "--L", "1200").c_str());
    to.drop = std::atof(arg(argc, argv, "--drop", "0").c_str());
    to.seed = std::strtoull(arg(argc, argv, "--seed", "1").c_str(), nullptr, 10);
    to.window = (uint32_t)std::atoi(arg(argc, argv, "--window", "64").c_str());
    to.header_version = std::atoi(arg(argc, argv, "--header-version", "0").c_str());
    to.device_mask = (uint32_t)std::strtoul(arg(argc, argv, "--device-mask", "0").c_str(), nullptr, 0);
    RxOptions ro;
    ro.ready = arg(argc, argv, "--ready", "ref") == "held" ? RxOptions::READY_HELD : RxOptions::READY_REFERENCE;
    ro.workers = std::atoi(arg(argc, argv, "--workers", "1").c_str());
    ro.ddl_ms = std::atoi(arg(argc, argv, "--ddl-ms", "50").c_str());
    ro.budget_bytes = std::strtoull(arg(argc, argv, "--budget", "0").c_str(), nullptr, 10);
    if (!ro.budget_bytes) ro.budget_bytes = 10ull << 20;
    ro.max_blocks = (uint32_t)std::atoi(arg(argc, argv, "--max-blocks", "128").c_str());
    ro.ring = (uint32_t)std::atoi(arg(argc, argv, "--ring", "4096").c_str());
    ro.device_mask = to.device_mask;
    const std::string transport = arg(argc, argv, "--transport", "inproc");
    const double timeout_s = std::atof(arg(argc, argv, "--timeout-s", "120").c_str());
    if (to.K == 0 || to.N < to.K || to.L == 0) { std::fprintf(stderr, "bad N/K/L\n"); return 2; }

    // file header (fileheader.go), computed by the sender
    struct stat stt;
    if (::stat(file.c_str(), &stt) != 0) { std::fprintf(stderr, "cannot stat %s\n", file.c_str()); return 2; }
    FileHeader fh;
    fh.file_size = (uint64_t)stt.st_size;
    fh.chunk_l = to.L;
    if (!sha256_file(file, fh.sha256)) return 2;
    uint8_t fhb[FILE_HEADER_LEN];
    marshal_file(fh, fhb);

    FileHeader rh;  // what the receiver read from its reliable channel
    int udp_rx = -1, udp_tx = -1;
    sockaddr_in ua{};
    if (transport == "udp") {
        // reliable channel: one TCP connection on 127.0.0.1 carries the file header
        const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in la{};
        la.sin_family = AF_INET;
        la.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        socklen_t sl = sizeof la;
        if (::bind(ls, (sockaddr*)&la, sizeof la) || ::listen(ls, 1) || ::getsockname(ls, (sockaddr*)&la, &sl)) {
            std::fprintf(stderr, "tcp setup failed\n");
            return 2;
        }
        std::thread cl([&] {
            const int c = ::socket(AF_INET, SOCK_STREAM, 0);
            if (::connect(c, (sockaddr*)&la, sizeof la) == 0) (void)!::write(c, fhb, sizeof fhb);
            ::close(c);
        });
        const int a = ::accept(ls, nullptr, nullptr);
        uint8_t got[FILE_HEADER_LEN];
        size_t n = 0;
        while (a >= 0 && n < sizeof got) {
            const ssize_t r = ::read(a, got + n, sizeof got - n);
            if (r <= 0) break;
            n += (size_t)r;
        }
        cl.join();
        ::close(a);
        ::close(ls);
        if (unmarshal_file(got, (uint32_t)n, &rh) != 0) { std::fprintf(stderr, "bad file header\n"); return 2; }
        udp_rx = ::socket(AF_INET, SOCK_DGRAM, 0);
        int rcv = 64 << 20;
        ::setsockopt(udp_rx, SOL_SOCKET, SO_RCVBUF, &rcv, sizeof rcv);
        timeval tv{0, 100000};
        ::setsockopt(udp_rx, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
        ua.sin_family = AF_INET;
        ua.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        sl = sizeof ua;
        if (::bind(udp_rx, (sockaddr*)&ua, sizeof ua) || ::getsockname(udp_rx, (sockaddr*)&ua, &sl)) return 2;
        udp_tx = ::socket(AF_INET, SOCK_DGRAM, 0);
        int snd = 16 << 20;
        ::setsockopt(udp_tx, SOL_SOCKET, SO_SNDBUF, &snd, sizeof snd);
        if (::connect(udp_tx, (sockaddr*)&ua, sizeof ua)) return 2;
    } else if (unmarshal_file(fhb, sizeof fhb, &rh) != 0) {
        return 2;
    }

    RxManager rx(rh.file_size, rh.chunk_l, out, ro);
    if (rx.start() != 0) { std::fprintf(stderr, "%s\n", rx.last_error().c_str()); return 2; }
    std::atomic<bool> rx_stop{false};
    std::thread net;
    if (udp_rx >= 0) {
        net = std::thread([&] {  // DATAGRAM receiver (transfer.go:382-411)
            constexpr int B = 64;
            std::vector<uint8_t> buf((size_t)B * 65536);
            mmsghdr msgs[B];
            iovec iov[B];
            while (!rx_stop.load() && rx.written() < rh.file_size) {
                for (int i = 0; i < B; ++i) {
                    iov[i].iov_base = buf.data() + (size_t)i * 65536;
                    iov[i].iov_len = 65536;
                    std::memset(&msgs[i].msg_hdr, 0, sizeof msgs[i].msg_hdr);
                    msgs[i].msg_hdr.msg_iov = &iov[i];
                    msgs[i].msg_hdr.msg_iovlen = 1;
                }
                const int n = ::recvmmsg(udp_rx, msgs, B, MSG_WAITFORONE, nullptr);
                for (int i = 0; i < n; ++i) deliver(rx, rh, buf.data() + (size_t)i * 65536, msgs[i].msg_len);
            }
        });
    }
    // --dump PATH: every datagram the sender emits, as [u32 length][bytes] records (tests compare the
    // symbols on the wire with the oracle's GenSymbol)
    const std::string dump_path = arg(argc, argv, "--dump", "");
    FILE* dump = dump_path.empty() ? nullptr : std::fopen(dump_path.c_str(), "wb");
    auto dump_dg = [&](const uint8_t* b, size_t n) {
        if (!dump) return;
        const uint32_t len = (uint32_t)n;
        std::fwrite(&len, 4, 1, dump);
        std::fwrite(b, 1, n, dump);
    };
    TxStats ts;
    const auto t0 = std::chrono::steady_clock::now();
    int rc;
    if (udp_tx >= 0) {
        rc = send_file(file, to, [&](const uint8_t* b, size_t n) {
            dump_dg(b, n);
            while (::send(udp_tx, b, n, 0) < 0 && errno == ENOBUFS) std::this_thread::yield();
        }, &ts);
    } else {
        // in-process datagrams with flow control: a full ingest ring makes the sender wait (as a
        // blocking socket would), so the only loss is the sender's --drop
        rc = send_file(file, to, [&](const uint8_t* b, size_t n) {
            dump_dg(b, n);
            while (rx.ring_full()) std::this_thread::sleep_for(std::chrono::microseconds(50));
            deliver(rx, rh, b, n);
        }, &ts);
    }
    if (dump) std::fclose(dump);
    // wait until the file is complete (transfer.go:349-359) or the timeout
    while (rc == 0 && rx.written() < rh.file_size &&
           std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < timeout_s)
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
    const double dur = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    rx_stop = true;
    if (net.joinable()) net.join();
    std::string final_path;
    const bool complete = rx.written() >= rh.file_size;
    const int fin = rx.close_and_finalize(rh.sha256, &final_path);
    if (udp_rx >= 0) ::close(udp_rx);
    if (udp_tx >= 0) ::close(udp_tx);
    char sh[65];
    hex(rh.sha256, sh);
    const RxStats& s = rx.stats;
    std::printf(
        "{\"ok\": %s, \"send_rc\": %d, \"complete\": %s, \"sha256_ok\": %s, \"sha256\": \"%s\", \"bytes\": %llu, "
        "\"dur_s\": %.4f, \"goodput_MBps\": %.2f, \"K\": %u, \"N\": %u, \"L\": %u, \"transport\": \"%s\", "
        "\"ready\": \"%s\", \"tx\": {\"dgrams\": %llu, \"bytes\": %llu, \"blocks\": %llu, \"dropped\": %llu, "
        "\"gpu_calls\": %llu, \"enc_ms\": %.2f, \"send_ms\": %.2f}, "
        "\"rx\": {\"dec_blocks\": %lld, \"gpu_calls\": %lld, \"gpu_decode_ms\": %.2f, \"fast_path_blocks\": %lld, "
        "\"decode_attempts\": %lld, \"decode_failures\": %lld, \"add_calls\": %lld, \"ready_blocks\": %lld, "
        "\"queued_ready\": %lld, \"queued_ddl\": %lld, \"dup\": %lld, \"drop_repairs\": %lld, \"drop_system\": %lld, "
        "\"ring_drop_r\": %lld, \"ring_drop_s\": %lld, \"budget_drop_r\": %lld, \"staging_drops\": %lld, "
        "\"write_ms\": %.2f, \"written\": %llu}, \"error\": \"%s\"}\n",
        (rc == 0 && complete && fin == 0) ? "true" : "false", rc, complete ? "true" : "false", fin == 0 ? "true" : "false",
        sh, (unsigned long long)rh.file_size, dur, rh.file_size / dur / 1e6, to.K, to.N, to.L, transport.c_str(),
        ro.ready == RxOptions::READY_HELD ? "held" : "ref", (unsigned long long)ts.dgrams, (unsigned long long)ts.bytes,
        (unsigned long long)ts.blocks, (unsigned long long)ts.dropped, (unsigned long long)ts.gpu_calls, ts.enc_s * 1e3,
        ts.send_s * 1e3, (long long)s.dec_blocks.load(), (long long)s.gpu_calls.load(), s.dec_us.load() / 1e3,
        (long long)s.fast_path_blocks.load(), (long long)s.decode_attempts.load(), (long long)s.decode_failures.load(),
        (long long)s.add_sym_count.load(), (long long)s.ready_blocks.load(), (long long)s.queued_by_ready.load(),
        (long long)s.queued_by_ddl.load(), (long long)s.dup_symbols.load(), (long long)s.drops_repairs.load(),
        (long long)s.drops_system.load(), (long long)s.ring_drop_repairs.load(), (long long)s.ring_drop_system.load(),
        (long long)s.budget_drop_repairs.load(), (long long)s.staging_drops.load(), s.write_us.load() / 1e3,
        (unsigned long long)rx.written(), rc ? rq_last_error() : rx.last_error().c_str());
    return (rc == 0 && complete && fin == 0) ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc >= 2 && std::strcmp(argv[1], "loopback") == 0) return loopback(argc, argv);
    std::fprintf(stderr, "usage: fecquic loopback --file F --out PATH [options]  (see fq_main.cpp)\n");
    return 2;
}
