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

}  // namespace rq
