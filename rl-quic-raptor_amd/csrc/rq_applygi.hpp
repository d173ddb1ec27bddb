// rq_applygi.hpp -- the register-table apply kernel's generator (rq_applygi.cpp).
#pragma once
#include <cstdint>
#include <string>

#include "rq_device.hpp"

namespace rq {

bool gi_shape_ok(const GiShape& sh);
uint32_t gi_vgprs(const GiShape& sh);
std::string gi_kernel_name(const GiShape& sh);
std::string emit_apply_gi_asm(const GiShape& sh);
// Static check of an apply kernel's text for shape sh (run on every generated kernel before assembly):
// while the VGPR index mode is on, the only vector instructions are the table lookups (a VOP2 XOR whose
// indexed first source is a table base, table + 2^G inside the allocation, into an accumulator outside
// the table); no vector-memory, LDS, branch or label inside an index-mode region; no instruction names
// M0 (it holds the mode's index and enable bits); every region is closed.  false + *err on a violation.
bool check_apply_gi_asm(const std::string& text, const GiShape& sh, std::string* err);

}  // namespace rq
