// rq_comgr.cpp -- in-process assembly of generated gfx950 code (amd_comgr): the column program's
// assembly text -> relocatable -> executable code object, ready for hipModuleLoadData.
// No subprocess: the library may run inside a process that already owns the GPU.
#include <amd_comgr/amd_comgr.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace rq {

namespace {
std::string log_of(amd_comgr_data_set_t set) {
    size_t n = 0;
    if (amd_comgr_action_data_count(set, AMD_COMGR_DATA_KIND_LOG, &n) != AMD_COMGR_STATUS_SUCCESS || n == 0) return {};
    amd_comgr_data_t d;
    if (amd_comgr_action_data_get_data(set, AMD_COMGR_DATA_KIND_LOG, 0, &d) != AMD_COMGR_STATUS_SUCCESS) return {};
    size_t sz = 0;
    std::string s;
    if (amd_comgr_get_data(d, &sz, nullptr) == AMD_COMGR_STATUS_SUCCESS) {
        s.resize(sz);
        amd_comgr_get_data(d, &sz, &s[0]);
    }
    amd_comgr_release_data(d);
    if (s.size() > 2000) s.resize(2000);
    return s;
}

// The generated code must stay inside the registers its descriptor allocates: an architectural VGPR
// at or above .amdhsa_accum_offset is an AGPR of the unified file (silently aliased, not rejected by
// the assembler), and an AGPR at or above next_free_vgpr - accum_offset is another wave's.
uint32_t directive(const std::string& src, const char* name) {
    const size_t at = src.find(name);
    return at == std::string::npos ? 0u : (uint32_t)std::strtoul(src.c_str() + at + std::strlen(name), nullptr, 10);
}

bool check_registers(const std::string& src, std::string* msg) {
    const uint32_t acc = directive(src, ".amdhsa_accum_offset"), total = directive(src, ".amdhsa_next_free_vgpr");
    if (!acc || !total || acc > total) { *msg += "no register allocation directives"; return false; }
    const size_t end = src.find(".amdhsa_kernel");
    auto ident = [](char c) { return std::isalnum((unsigned char)c) || c == '_' || c == '.'; };
    for (size_t i = 1; i < std::min(end, src.size()); ++i) {
        const char c = src[i];
        if ((c != 'v' && c != 'a') || ident(src[i - 1])) continue;
        size_t j = i + 1;
        if (j < src.size() && src[j] == '[') ++j;  // v[a:b]: the upper end is checked below
        if (j >= src.size() || !std::isdigit((unsigned char)src[j])) continue;
        uint32_t r = (uint32_t)std::strtoul(src.c_str() + j, nullptr, 10);
        while (j < src.size() && std::isdigit((unsigned char)src[j])) ++j;
        if (src[i + 1] == '[' && j < src.size() && src[j] == ':') r = (uint32_t)std::strtoul(src.c_str() + j + 1, nullptr, 10);
        else if (src[i + 1] != '[' && j < src.size() && ident(src[j])) continue;
        const uint32_t lim = c == 'v' ? acc : total - acc;
        if (r >= lim) {
            *msg += std::string("register ") + c + std::to_string(r) + " beyond the allocation (" + std::to_string(lim) + ")";
            return false;
        }
    }
    return true;
}
}  // namespace

bool comgr_assemble(const std::string& src, std::vector<char>* co, std::string* err) {
    {
        std::string m = "comgr: ";
        if (!check_registers(src, &m)) {
            if (err) *err = m;
            return false;
        }
    }
    amd_comgr_data_t in_d{};
    amd_comgr_data_set_t in{}, reloc{}, exe{};
    amd_comgr_action_info_t ai{};
    bool ok = false;
    std::string msg = "comgr: ";
    do {
        if (amd_comgr_create_data(AMD_COMGR_DATA_KIND_SOURCE, &in_d) != AMD_COMGR_STATUS_SUCCESS) { msg += "create_data"; break; }
        if (amd_comgr_set_data(in_d, src.size(), src.data()) != AMD_COMGR_STATUS_SUCCESS ||
            amd_comgr_set_data_name(in_d, "colprog.s") != AMD_COMGR_STATUS_SUCCESS) { msg += "set_data"; break; }
        if (amd_comgr_create_data_set(&in) != AMD_COMGR_STATUS_SUCCESS ||
            amd_comgr_data_set_add(in, in_d) != AMD_COMGR_STATUS_SUCCESS ||
            amd_comgr_create_data_set(&reloc) != AMD_COMGR_STATUS_SUCCESS ||
            amd_comgr_create_data_set(&exe) != AMD_COMGR_STATUS_SUCCESS) { msg += "data sets"; break; }
        if (amd_comgr_create_action_info(&ai) != AMD_COMGR_STATUS_SUCCESS ||
            amd_comgr_action_info_set_isa_name(ai, "amdgcn-amd-amdhsa--gfx950") != AMD_COMGR_STATUS_SUCCESS ||
            amd_comgr_action_info_set_logging(ai, true) != AMD_COMGR_STATUS_SUCCESS) { msg += "action info"; break; }
        if (amd_comgr_do_action(AMD_COMGR_ACTION_ASSEMBLE_SOURCE_TO_RELOCATABLE, ai, in, reloc) != AMD_COMGR_STATUS_SUCCESS) {
            msg += "assemble failed: " + log_of(reloc);
            break;
        }
        if (amd_comgr_do_action(AMD_COMGR_ACTION_LINK_RELOCATABLE_TO_EXECUTABLE, ai, reloc, exe) != AMD_COMGR_STATUS_SUCCESS) {
            msg += "link failed: " + log_of(exe);
            break;
        }
        amd_comgr_data_t od;
        if (amd_comgr_action_data_get_data(exe, AMD_COMGR_DATA_KIND_EXECUTABLE, 0, &od) != AMD_COMGR_STATUS_SUCCESS) {
            msg += "no executable";
            break;
        }
        size_t sz = 0;
        if (amd_comgr_get_data(od, &sz, nullptr) == AMD_COMGR_STATUS_SUCCESS) {
            co->resize(sz);
            ok = amd_comgr_get_data(od, &sz, co->data()) == AMD_COMGR_STATUS_SUCCESS;
        }
        amd_comgr_release_data(od);
        if (!ok) msg += "get_data";
    } while (false);
    if (ai.handle) amd_comgr_destroy_action_info(ai);
    if (exe.handle) amd_comgr_destroy_data_set(exe);
    if (reloc.handle) amd_comgr_destroy_data_set(reloc);
    if (in.handle) amd_comgr_destroy_data_set(in);
    if (in_d.handle) amd_comgr_release_data(in_d);
    if (!ok && err) *err = msg;
    return ok;
}

}  // namespace rq
