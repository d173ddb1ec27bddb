// rq_comgr.cpp -- in-process assembly of generated gfx950 code (amd_comgr): the column program's
// assembly text -> relocatable -> executable code object, ready for hipModuleLoadData.
// No subprocess: the library may run inside a process that already owns the GPU.
#include <amd_comgr/amd_comgr.h>

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
}  // namespace

bool comgr_assemble(const std::string& src, std::vector<char>* co, std::string* err) {
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
