/*
 * drop_in_caller.c -- TEST PROGRAM: a compiled caller of libtrpo_mi355x.so through the reference's own
 * entry points, the way src/TRPOCpuCode.c drives src/TRPO_FVP.c / TRPO_CG.c / TRPO_Update.c
 * (Test_FVP / Test_CG at src/TRPOCpuCode.c:15-135, Test_TRPO_Update at :314-372): a TRPOparam filled
 * field by field and passed BY VALUE, caller-owned fp64 vectors, the "< 0 means failure" return
 * convention.  Built by tests/c_caller/Makefile as C (gcc) and as C++ (g++, as the reference's
 * build/Makefile.cpuonly compiles its callers) against include/trpo_mi355x.h -- C++ both with the C
 * names and with TRPO_MI355X_CXX_LINKAGE (the mangled names an unchanged g++ caller imports) -- and,
 * where /root/reference exists, as C++ against the reference's OWN src/include/TRPO.h
 * (-DUSE_REFERENCE_HEADER): the unchanged-caller case of build/Makefile.cpuonly:5,11.
 *
 *   drop_in_caller FIXTURE_DIR OUT_DIR [NumSamples [NumThreads]]
 *
 * Reads ArmTestModel.txt / ArmTestData.txt / ArmTestFVP.txt / ArmTestCG.txt from FIXTURE_DIR and writes
 * OUT_DIR/fvp.txt (FVPFast of ArmTestFVP.txt column 1), OUT_DIR/cg.txt (CG(10, 1e-10) of ArmTestCG.txt
 * column 1) and OUT_DIR/update.txt (TRPO_Update), one %.17g value per line.  The library itself prints
 * the reference's stdout lines (CG Iter[...], shs, lagrange multiplier, a/e/r).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef USE_REFERENCE_HEADER
#include "TRPO.h"
#else
#include "trpo_mi355x.h"
#endif

static int read_column(const char *path, int col, double *v, size_t n) {
    FILE *f = fopen(path, "r");
    if (!f) {
        fprintf(stderr, "[ERROR] Cannot open Data File [%s]. \n", path);
        return -1;
    }
    for (size_t i = 0; i < n; ++i) {
        double a, b;
        if (fscanf(f, "%lf %lf", &a, &b) != 2) {
            fclose(f);
            return -1;
        }
        v[i] = col == 0 ? a : b;
    }
    fclose(f);
    return 0;
}

static int write_vector(const char *dir, const char *name, const double *v, size_t n) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE *f = fopen(path, "w");
    if (!f) return -1;
    for (size_t i = 0; i < n; ++i) fprintf(f, "%.17g\n", v[i]);
    fclose(f);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s FIXTURE_DIR OUT_DIR [NumSamples [NumThreads]]\n", argv[0]);
        return 2;
    }
    const char *dir = argv[1], *out = argv[2];
    const size_t num_samples = argc > 3 ? (size_t)strtoull(argv[3], NULL, 10) : 3150;
    const size_t num_threads = argc > 4 ? (size_t)strtoull(argv[4], NULL, 10) : 6;

    /* ArmDOF_0-v0 */
    char AcFunc[] = {'l', 't', 't', 'l'};
    size_t LayerSize[] = {15, 16, 16, 3};
    char model[4096], data[4096], fvpfile[4096], cgfile[4096];
    snprintf(model, sizeof model, "%s/ArmTestModel.txt", dir);
    snprintf(data, sizeof data, "%s/ArmTestData.txt", dir);
    snprintf(fvpfile, sizeof fvpfile, "%s/ArmTestFVP.txt", dir);
    snprintf(cgfile, sizeof cgfile, "%s/ArmTestCG.txt", dir);

    TRPOparam Param;
    memset(&Param, 0, sizeof Param);
    Param.ModelFile = model;
    Param.DataFile = data;
    Param.NumLayers = 4;
    Param.AcFunc = AcFunc;
    Param.LayerSize = LayerSize;
    Param.NumSamples = num_samples;
    Param.CG_Damping = 0.1;

    const size_t P = NumParamsCalc(Param.LayerSize, Param.NumLayers);
    double *input = (double *)calloc(P, sizeof(double));
    double *result = (double *)calloc(P, sizeof(double));
    if (!input || !result) return 3;
    int failed = 0;

    if (read_column(fvpfile, 0, input, P)) return 4;
    double t = FVPFast(Param, result, input, num_threads);
    if (t < 0) {
        fprintf(stderr, "[ERROR] Fisher Vector Product Calculation Failed.\n");
        failed = 1;
    } else {
        printf("[INFO] FVPFast (%zu Threads) Computing Time = %f seconds\n", num_threads, t);
        failed |= write_vector(out, "fvp.txt", result, P) != 0;
    }

    if (read_column(cgfile, 0, input, P)) return 4;
    t = CG(Param, result, input, 10, 1e-10, num_threads);
    if (t < 0) {
        fprintf(stderr, "[ERROR] Conjugate Gradient Calculation Failed.\n");
        failed = 1;
    } else {
        printf("[INFO] CG Computing Time = %f seconds\n", t);
        failed |= write_vector(out, "cg.txt", result, P) != 0;
    }

    t = TRPO_Update(Param, result, num_threads);
    if (t < 0) {
        fprintf(stderr, "[ERROR] TRPO Update Failed.\n");
        failed = 1;
    } else {
        printf("[INFO] TRPO_Update Computing Time = %f seconds\n", t);
        failed |= write_vector(out, "update.txt", result, P) != 0;
    }

    /* a bad path must come back as -1 with the reference's message, not crash */
    char missing[] = "/nonexistent/ArmTestModel.txt";
    Param.ModelFile = missing;
    if (FVPFast(Param, result, input, num_threads) >= 0) failed = 1;

    free(input);
    free(result);
    return failed;
}
