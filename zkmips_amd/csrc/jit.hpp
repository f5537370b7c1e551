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
    hipFunction_t fn = nullptr;
    std::vector<char> code;
};

bool jit_enabled();
std::vector<char> jit_quotient_code(const ChipDesc &c, const std::string &arch_name);
JitKernel jit_quotient(const ChipDesc &c, int device);
void launch_quotient_jit(const JitKernel &k, const ZkmQuotJitArgs &a, hipStream_t s);

}  // namespace zkm
