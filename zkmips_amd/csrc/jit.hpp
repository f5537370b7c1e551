// JIT-specialised quotient kernels (see jit.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "chip.hpp"
#include "jit_abi.h"

namespace zkm {

struct JitKernel {
    bool ok = false;
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;       // quotient
    hipFunction_t fn_perm = nullptr;  // permutation trace rows (chips with local lookups)
    std::vector<char> code;
};

bool jit_enabled();
std::vector<char> jit_chip_code(const ChipDesc &c, const std::string &arch_name);
JitKernel jit_chip(const ChipDesc &c, int device);
void launch_quotient_jit(const JitKernel &k, const ZkmQuotJitArgs &a, hipStream_t s);
void launch_perm_jit(const JitKernel &k, const ZkmPermJitArgs &a, hipStream_t s);

}  // namespace zkm
