// rq_colprog.hpp -- the "column program": RaptorQ encode compiled to straight-line gfx950 code.
//
// One GPU lane owns one dword column (4 bytes) of one source block; all lanes run the same
// program, which depends only on (K', K, the requested output symbols).  The program computes
// the requested repair symbols of the constraint system A*C = D that xssnick's Solve handles per
// block (RQ/solver.go:25-185), without ever materialising C:
//
//   forward pass  y_k = D_row(k) ^ XOR_{j in deps(k)} y_j       (peeling order, RQ/inactivate.go)
//   Horner scan   bh = G_HDPC * y  (MT * Gamma, RQ/params.go:116-133) in column order, which also
//                 pushes every y into the remaining-row sums b2 and the output sums
//   dense part    C_F = Zi*bh ^ Q*b2  (H values; GF(256) by bit-decomposed Horner: xtime + XOR)
//   outputs       out_j = XOR_{c in LT(j), pivoted} y_c ^ V1_j*b2 ^ V2_j*C_F   (encodeGen,
//                 RQ/params.go:162-182, with C = y ^ W*C_U folded in)
//
// C is the unique solution of a full-rank system, so the outputs are
// bit-exact with the reference whatever elimination order is used here.  Every operation is an
// XOR of 2-3 values or a multiply by alpha (xtime) -- no general GF(256) multiply survives.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

#include "rq_core.hpp"

namespace rq {

// Experiment knobs (RQHIP_DIAG, RQHIP_ALLOC, RQHIP_POLICY, ...: tuning sweeps and diagnostic modes,
// some of which produce wrong bytes on purpose) are read only in builds made with
// `make EXPERIMENTS=1`; the shipped library ignores the environment.
inline const char* knob(const char* name) {
#ifdef RQHIP_EXPERIMENTS
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

enum IrKind : uint8_t {
    IR_LOAD = 0,  // imm = source row (< K)
    IR_ZERO = 1,
    IR_XOR2 = 2,  // a ^ b
    IR_XOR3 = 3,  // a ^ b ^ c
    IR_XT = 4,    // alpha * a (per byte, GF(256) poly 0x11D)
    IR_XTX = 5,   // alpha * a ^ b
    IR_STORE = 6,  // output imm <- a
    // two-wave (pair) programs only (split_pair): the hand-off between the waves through an LDS ring
    IR_SEND = 7,   // ring slot imm <- a (wave A)
    IR_RECV = 8,   // value <- ring slot imm (wave B)
    IR_BAR = 9     // workgroup barrier closing a transfer (imm = transfer index)
};
constexpr uint32_t NOVAL = 0xFFFFFFFFu;
// build_colprog's `passes` with this bit set: replacement-selection Horner runs with a buffer of
// (passes & 0xFFFF) produced y values (see build() in rq_colprog.cpp).
constexpr uint32_t SCHED_RS = 1u << 16;
// ... with this bit set instead: no Horner scan, bh accumulated bit by bit over groups of produced y.
constexpr uint32_t SCHED_4R = 1u << 17;
// ... and (SCHED_4R only) bits 20..27 = n: the first n HDPC rows' bit accumulation tagged grp 4 with
// their own subset sums (split_pair then runs them on wave A unless bmask has bit 4).
constexpr uint32_t SCHED_HA_SHIFT = 20;

struct IrNode {
    uint8_t k = IR_ZERO;
    uint32_t a = NOVAL, b = NOVAL, c = NOVAL;  // operand value ids (node indices)
    uint32_t imm = 0;
    // what the node computes (SCHED_4R programs; split_pair assigns waves by it): 0 forward pass
    // (peeling: y values and their pushes into dependent rows), 1 HDPC bit accumulation (subset sums,
    // bit rows, bh), 2 pushes into the remaining-row and output sums (and b2), 3 dense part and outputs,
    // 4 the bit accumulation of the HDPC rows given to wave A (SCHED_HA_SHIFT)
    uint8_t grp = 0;
};

struct ColIR {
    Params p{};
    std::vector<IrNode> nodes;     // program order; node i defines value i (except STORE)
    uint32_t n_out = 0;
    uint32_t phase_start[4] = {0, 0, 0, 0};  // forward, scan, dense, outputs
    struct Stats {
        uint32_t xor2 = 0, xor3 = 0, xt = 0, xtx = 0, load = 0, store = 0, zero = 0;
        uint32_t u = 0, npiv = 0, n2 = 0;
        uint32_t push_dep = 0, push_rem = 0, push_out = 0;  // SCHED_4R production pushes by target
    } st;
};

// Outputs are ESIs with the library's GenSymbol meaning (RQ/encoder.go:36-41): esi < K is the
// zero-padded source row, otherwise the LT symbol of ISI esi + K' - K.  p.K is the library K.
// passes: 0 = one demand-driven column scan; P >= 1 = peeling-order production with P Horner passes
// (see build() in rq_colprog.cpp).  Every choice computes the same bytes.
bool build_colprog(const Params& p, const uint32_t* esi, uint32_t n_out, ColIR* ir, std::string* err,
                   uint32_t passes = 0);
// Outputs are the L intermediate symbols C[0..L-1] (per-object encoder: GenSymbol gathers).
bool build_colprog_C(const Params& p, ColIR* ir, std::string* err, uint32_t passes = 0);
// Two-wave split of a column program (one workgroup of two waves per item, one wave per SIMD):
// wave A runs the nodes whose grp is not in bmask -- every source load, the forward pass, the pushes
// -- and wave B the others (the HDPC bit accumulation, the dense part and the outputs), so B's VALU
// work never waits behind A's memory instructions in one in-order issue stream.  Every A value that
// B uses goes through a ring of LDS slots in transfers of at most max_xfer values, each closed by a
// workgroup barrier; B runs `lag` transfers behind A (B starts with `lag` barriers, A ends with
// them).  No B value may feed an A node.
struct PairIR {
    ColIR A, B;
    uint32_t lag = 0;
    uint32_t ring = 0;       // ring slots (256 B each) at the start of the workgroup's LDS
    uint32_t n_xfer = 0;     // transfers per item (= barriers per item on each side)
    uint32_t n_cross = 0;    // values handed from A to B per item
    uint32_t max_window = 0; // most slots in use at once (lag + 2 consecutive transfers)
};
bool split_pair(const ColIR& ir, uint32_t bmask, uint32_t lag, uint32_t max_xfer, uint32_t ring, PairIR* out,
                std::string* err);

// Host evaluation of the IR on one block (test reference for the compiler, not a product path):
// src = K rows x T bytes, out = n_out rows x T bytes.
void eval_colprog(const ColIR& ir, const uint8_t* src, uint32_t T, uint8_t* out);

}  // namespace rq
