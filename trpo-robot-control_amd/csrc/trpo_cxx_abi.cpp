/*
 * trpo_cxx_abi.cpp -- the C++-linkage face of the drop-in entry points.
 *
 * The reference declares its L3 core in src/include/TRPO.h:81-104 WITHOUT extern "C", and its CPU
 * build (build/Makefile.cpuonly:5,11) compiles every caller -- TRPOCpuCode.c, the trainers -- with
 * g++ -std=c++11.  An unchanged caller therefore imports the Itanium-mangled symbols
 * (_Z7FVPFast9TRPOparamPdS0_m, _Z2CG9TRPOparamPdS0_mdm, _Z13NumParamsCalcPmm, ...), not the C names.
 * This translation unit defines exactly those C++ functions (same parameter types: the typedef'd
 * anonymous TRPOparam mangles by its typedef name) and forwards each to the C export of
 * csrc/trpo_host.c, so the library serves C callers and unchanged g++-built callers alike.
 *
 *   TRPO.h:81  NumParamsCalc   TRPO.h:89  FVP        TRPO.h:93  FVPFast    TRPO.h:96  CG
 *   TRPO.h:98  FVP_FPGA        TRPO.h:101 CG_FPGA    TRPO.h:104 TRPO_Update
 *
 * evaluate() needs no twin: src/include/lbfgs.h:32-34 gives the liblbfgs callback C linkage.
 * The C functions are reached through asm labels (a C-linkage declaration under another source name),
 * since one scope cannot declare the same name with both linkages.
 */
#define TRPO_MI355X_CXX_LINKAGE
#include "trpo_mi355x.h"

extern "C" {
size_t c_NumParamsCalc(size_t *, size_t) __asm__("NumParamsCalc");
double c_FVP(TRPOparam, double *, double *) __asm__("FVP");
double c_FVPFast(TRPOparam, double *, double *, size_t) __asm__("FVPFast");
double c_CG(TRPOparam, double *, double *, size_t, double, size_t) __asm__("CG");
double c_FVP_FPGA(TRPOparam, double *, double *) __asm__("FVP_FPGA");
double c_CG_FPGA(TRPOparam, double *, double *, size_t, double, size_t) __asm__("CG_FPGA");
double c_TRPO_Update(TRPOparam, double *, size_t) __asm__("TRPO_Update");
}

#define EXPORT __attribute__((visibility("default")))

EXPORT size_t NumParamsCalc(size_t *LayerSize, size_t NumLayers) { return c_NumParamsCalc(LayerSize, NumLayers); }

EXPORT double FVP(TRPOparam param, double *Result, double *Input) { return c_FVP(param, Result, Input); }

EXPORT double FVPFast(TRPOparam param, double *Result, double *Input, size_t NumThreads) {
    return c_FVPFast(param, Result, Input, NumThreads);
}

EXPORT double CG(TRPOparam param, double *Result, double *b, size_t MaxIter, double ResidualTh, size_t NumThreads) {
    return c_CG(param, Result, b, MaxIter, ResidualTh, NumThreads);
}

EXPORT double FVP_FPGA(TRPOparam param, double *Result, double *Input) { return c_FVP_FPGA(param, Result, Input); }

EXPORT double CG_FPGA(TRPOparam param, double *Result, double *b, size_t MaxIter, double ResidualTh,
                      size_t NumThreads) {
    return c_CG_FPGA(param, Result, b, MaxIter, ResidualTh, NumThreads);
}

EXPORT double TRPO_Update(TRPOparam param, double *Result, size_t NumThreads) {
    return c_TRPO_Update(param, Result, NumThreads);
}
