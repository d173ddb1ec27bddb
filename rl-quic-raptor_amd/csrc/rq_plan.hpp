// rq_plan.hpp -- per-K' encode schedule ("plan") compiler.
//
// The reference solves A*C = D for every block from scratch (xssnick Solve, RQ/solver.go:25-185:
// inactivation decoding RQ/inactivate.go:25-170, GF(2) block products, hdpcMultiply
// RQ/params.go:116-133, GaussianElimination RQ/discmath/gauss.go:7-45).  For encode the
// constraint matrix depends only on K' (SURVEY.md sec. 0.5), so rqhip runs that elimination ONCE
// per K' on the coefficient matrix only and records the symbol operations as a straight-line
// program over "slots" (rows of a column strip held in LDS).  The GPU replays the program on
// every (block, strip).  C is the unique solution of a full-rank system, so
// the replay is bit-exact with the reference whatever elimination order the compiler picks.
//
// Program shape (all phases emit statements; a list scheduler packs independent statements
// into levels separated by workgroup barriers):
//   load   : slot(row of ISI i) <- source symbol i (zero for i >= K or erased), others zero
//   pass A : forward substitution over peeled LT/LDPC rows, y in place (XOR)
//   rest   : remaining GF(2) rows reduced by y (XOR)
//   hdpc   : HDPC right-hand sides via chunked Horner over MT*Gamma (xtime + XOR per column)
//   dense  : u x u solve on the inactive columns (GF(2) RREF, H x (u-H) mul-adds, H x H solve)
//   pass B : final C of peeled columns: y ^ W*C_U (in place) or source reload ^ deps ^ rowU
//   output : LT gathers (repair symbols = XOR of C rows, RQ/params.go:162-182) -> global
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "rq_core.hpp"

namespace rq {

enum StmtType : uint32_t {
    ST_XOR = 0,     // dst = (ACC ? dst : 0) ^ XOR_k src_k
    ST_MUL = 1,     // dst = (ACC ? dst : 0) ^ SUM_k c_k * src_k            (GF(256))
    ST_SCALE = 3,   // dst = c * dst                                        (c in word 1)
    ST_HORNER = 4,  // HDPC chunk: see rq_kernels.hip
};
constexpr uint32_t ST_FLAG_ACC = 1u << 31;
constexpr uint32_t SRC_GLOBAL = 1u << 31;   // source word: re-read source row (isi in low 24 bits)
constexpr uint16_t SLOT_NONE = 0xFFFF;

// Statement word 0: dst(16) | nsrc(12) | type(3) | ACC(1).  Then (SCALE) one extra word,
// then nsrc source words: slot(16) | coef(8) | 0, or SRC_GLOBAL | isi for a source row that is
// re-read from global memory (zero if isi >= K or erased).  HORNER: word0 dst = first of H
// partial slots, nsrc = chunk length; per column word: slot(16) | a(5) | b(5) -- t is added to
// partials a and b (a == b: nothing); then ceil(H/4) words of tau coefficients (partial[h] ^=
// tau_h * t at the end of the chunk; the last chunk's tau includes MT[h][KS-1] = alpha^h).
struct Stmt {
    uint32_t type = ST_XOR;
    bool acc = false;
    uint16_t dst = 0;
    uint32_t extra = 0;
    uint32_t phase = 0;          // 0 passA 1 rest 2 horner 3 hdpcsum 4 D1 5 D2 6 D3 7 passB
    std::vector<uint32_t> src;   // encoded source words
};

struct PlanStats {
    uint32_t n_stmts = 0, n_levels = 0, n_src_xor = 0, n_src_mul = 0, n_reload = 0;
    uint32_t u = 0, inactivated = 0, n_pivots = 0, n_slots = 0, max_level_width = 0;
    uint32_t horner_chunks = 0, passB_inplace = 0, passB_reload = 0;
    uint32_t phase_lo[8] = {0}, phase_hi[8] = {0}, phase_n[8] = {0};
};

struct Plan {
    Params p{};
    uint32_t n_slots = 0;                 // L + temporaries
    std::vector<uint16_t> load_slot;      // [K'] slot receiving source/pad row i
    std::vector<uint16_t> col_slot;       // [L]  slot holding C[c] at program end
    std::vector<uint32_t> level_start;    // [n_levels + 1] statement index ranges
    std::vector<uint32_t> stmt_off;       // [n_stmts + 1] offsets into words
    std::vector<uint32_t> words;          // encoded statements in level order
    PlanStats stats;
};

// Compile the encode plan for the parameter row of K (K' = p.Kp).  Returns false (and sets
// *err) if the constraint matrix is singular (never expected for RFC 6330 rows).
struct PlanOptions {
    uint32_t horner_chunks = 16;  // parallel chunks of the HDPC Horner scan
    uint32_t depth_a = 1u << 30;  // dependency-depth cap of the forward substitution (pass A)
    uint32_t depth_b = 1u << 30;  // dependency-depth cap of the final substitution (pass B)
    // pass B: 1 = in place only (C_k = y_k ^ W_k C_U: one level, no source re-reads from global
    // memory); 0 = per row the cheaper of in place / rebuild (fewer XORs, ~90 more levels)
    uint32_t passb_mode = 1;
};
bool compile_encode_plan(const Params& p, Plan* out, std::string* err, const PlanOptions& opt = PlanOptions());

// ---------------------------------------------------------------------------------------
// Wave program: the level-scheduled statements re-packed into per-wave instruction streams for
// k_encode; the stream format is specified in rq_wave_format.hpp.
struct WaveProgram {
    uint32_t n_waves = 0, n_levels = 0, n_slots = 0, zero_slot = 0, trash_slot = 0, sd = 0;
    std::vector<uint32_t> words;      // all streams, padded for chunk prefetch
    std::vector<uint32_t> wave_off;   // [n_waves] stream start
    uint32_t max_stream = 0;          // longest stream (words)
};
// Slot fields are LDS byte offsets (slot * sd * 4) for a strip of sd dwords (sd > 0).
bool build_wave_program(const Plan& plan, uint32_t n_waves, uint32_t sd, WaveProgram* out, std::string* err);

// Encode the output (LT gather) statements for a list of ISIs: per output one word
// nsrc(8) followed by nsrc slots (C columns mapped through col_slot).  Appended to *words;
// returns the offset of each output in *offs.
void encode_outputs(const Plan& plan, const uint32_t* isi, uint32_t n, std::vector<uint32_t>* words,
                    std::vector<uint32_t>* offs);

}  // namespace rq
