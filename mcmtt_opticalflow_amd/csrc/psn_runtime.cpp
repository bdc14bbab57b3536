// One HIP / HSA / RCCL / comgr runtime per process.
//
// libpsn_lk.so links the ROCm runtime by soname (libamdhip64.so.7,
// libhsa-runtime64.so.1, librccl.so.1; RUNPATH /opt/rocm/lib). PyTorch-ROCm
// ships its own copies of the same libraries and its libraries ask for them by
// the UNVERSIONED names (libc10_hip.so: NEEDED libamdhip64.so, RPATH $ORIGIN).
// The dynamic loader matches a NEEDED name against a loaded object's soname or
// the names it was loaded under, so when this library loads first and torch
// second, "libamdhip64.so" matches nothing, torch's copy is mapped beside ours,
// and the second HIP/HSA runtime's init fails ("No HIP GPUs are available").
//
// At load time this library gives the runtime objects it is bound to their
// unversioned names as well: dlopen(<unversioned>, RTLD_NOLOAD) finds the same
// file (same inode) through our RUNPATH and glibc adds the name to the loaded
// object, or finds a different file and maps nothing. A library loaded later
// that asks for the unversioned name then binds to the same runtime. When torch
// was loaded first, our sonames already resolve to torch's copies and the
// unversioned names are already theirs: one runtime either way, whichever loads
// first. comgr (which the HIP runtime dlopens lazily by soname) is mapped here
// from the same directory so a later torch import cannot supply its own.
// psn_lk_runtime_info() reports the files that were bound.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>

#include "psn_lk.h"

namespace {

struct RuntimeName {
    const char *soname;      // what this library (or the HIP runtime) asks for
    const char *unversioned; // what torch's libraries ask for
};

const RuntimeName kRuntimes[] = {
    {"libamdhip64.so.7", "libamdhip64.so"},
    {"libhsa-runtime64.so.1", "libhsa-runtime64.so"},
    {"librccl.so.1", "librccl.so"},
    {"libamd_comgr.so.3", "libamd_comgr.so"},
};

int g_aliased = 0;  // bit i: kRuntimes[i]'s unversioned name now resolves to the bound object

__attribute__((constructor)) void bind_runtime_names() {
    for (int i = 0; i < (int)(sizeof(kRuntimes) / sizeof(kRuntimes[0])); i++) {
        // searched with this library's RUNPATH; already mapped for the first three
        void *h = dlopen(kRuntimes[i].soname, RTLD_LAZY | RTLD_LOCAL);
        if (!h) continue;
        void *a = dlopen(kRuntimes[i].unversioned, RTLD_LAZY | RTLD_LOCAL | RTLD_NOLOAD);
        if (a == h) g_aliased |= 1 << i;  // (glibc: a handle is the object's link map)
        // both handles stay open for the life of the process
    }
}

const char *path_of(const void *sym) {
    Dl_info di{};
    if (sym && dladdr(sym, &di) && di.dli_fname) return di.dli_fname;
    return "";
}

}  // namespace

extern "C" int psn_lk_runtime_info(char *buf, int len) {
    if (!buf || len <= 0) return PSN_LK_ERR_ARG;
    int hip_rt = 0;
    (void)hipRuntimeGetVersion(&hip_rt);  // no device init
    int nccl = 0;
    (void)ncclGetVersion(&nccl);
    void *comgr = dlopen(kRuntimes[3].soname, RTLD_LAZY | RTLD_LOCAL | RTLD_NOLOAD);
    void *comgr_sym = comgr ? dlsym(comgr, "amd_comgr_get_version") : nullptr;
    int n = snprintf(buf, (size_t)len,
                     "{\"libamdhip64\": \"%s\", \"libhsa-runtime64\": \"%s\", \"librccl\": \"%s\", "
                     "\"libamd_comgr\": \"%s\", \"hip_runtime_version\": %d, \"rccl_version\": %d, "
                     "\"unversioned_names_bound\": %d, \"built_against_hip\": %d}",
                     path_of((const void *)&hipRuntimeGetVersion), path_of((const void *)&hsa_init),
                     path_of((const void *)&ncclGetVersion), path_of(comgr_sym), hip_rt, nccl, g_aliased,
                     HIP_VERSION);
    if (comgr) dlclose(comgr);
    return n < len ? PSN_LK_OK : PSN_LK_ERR_ARG;
}
