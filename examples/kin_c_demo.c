/* kin_c_demo.c -- the C-ABI from plain C (no Python, no C++): what a Julia ccall / cgo /
 * JNI binding does.  Parses fetch.urdf with the native loader, plans FK + 6x8 Jacobian of
 * gripper_link over the 8 arm joints, specialises the plan, runs N configurations (q = 0 for
 * the first, random for the rest) on the device, and checks the q = 0 pose against the value
 * the reference gives (gripper_link at q = 0 -> (1.1281, 0, 0.78601)) and the
 * angular Jacobian rows against unit axes.
 * Build: gcc -O2 -std=c11 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude examples/kin_c_demo.c
 *        -Lkinematics.jl_amd/lib -lkinhip -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,... -lm */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "kinhip.h"

#define CK(x)                                                                                \
    do {                                                                                     \
        int rc_ = (x);                                                                       \
        if (rc_ != 0) {                                                                      \
            fprintf(stderr, "%s failed: %d %s\n", #x, rc_, kin_last_error() ? kin_last_error() : ""); \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

int main(int argc, char** argv) {
    if (kin_abi_version() != KINHIP_ABI_VERSION) {  /* the kin_* structs this file was compiled against */
        fprintf(stderr, "libkinhip C-ABI version %d, this program needs %d\n", kin_abi_version(), KINHIP_ABI_VERSION);
        return 1;
    }
    const char* urdf = argc > 1 ? argv[1] : "tests/golden/fetch.urdf";
    const char* arm[8] = {"torso_lift_joint", "shoulder_pan_joint", "shoulder_lift_joint", "upperarm_roll_joint",
                          "elbow_flex_joint", "forearm_roll_joint", "wrist_flex_joint", "wrist_roll_joint"};
    kin_urdf* u;
    CK(kin_urdf_parse_file(urdf, &u));
    kin_tree_desc d;
    CK(kin_urdf_tree(u, 0, &d));
    kin_model* m;
    CK(kin_model_create(&d, &m));
    int32_t ids[8], gl;
    for (int k = 0; k < 8; ++k) CK(kin_urdf_find_joint(u, arm[k], &ids[k]));
    CK(kin_urdf_find_link(u, "gripper_link", &gl));
    kin_plan_desc pd = {KIN_F32, 8, ids, 1, &gl, gl, 8, ids, KIN_WITH_ROT | KIN_ZERO_FILL};
    kin_plan* p;
    CK(kin_plan_create(m, &pd, &p));
    CK(kin_plan_specialize(p, KIN_SPEC_FK));
    const int64_t N = 4096;
    float* hq = (float*)malloc(sizeof(float) * 8 * N);
    srand(7);
    for (int64_t i = 0; i < 8 * N; ++i) hq[i] = (i % N == 0) ? 0.0f : (float)rand() / RAND_MAX - 0.5f;
    float *dq, *dp, *dj;
    if (hipMalloc((void**)&dq, sizeof(float) * 8 * N) || hipMalloc((void**)&dp, sizeof(float) * 12 * N) ||
        hipMalloc((void**)&dj, sizeof(float) * 48 * N))
        return 1;
    if (hipMemcpy(dq, hq, sizeof(float) * 8 * N, hipMemcpyHostToDevice)) return 1;
    CK(kin_plan_run(p, dq, N, N, dp, N, dj, N, NULL));
    float* hp = (float*)malloc(sizeof(float) * 12 * N);
    float* hj = (float*)malloc(sizeof(float) * 48 * N);
    if (hipMemcpy(hp, dp, sizeof(float) * 12 * N, hipMemcpyDeviceToHost) ||
        hipMemcpy(hj, dj, sizeof(float) * 48 * N, hipMemcpyDeviceToHost))
        return 1;
    const double x = hp[9 * N], y = hp[10 * N], z = hp[11 * N];
    double worst = 0;
    for (int64_t i = 0; i < N; ++i)
        for (int c = 1; c < 8; ++c) {  // revolute columns: rows 4:6 are unit world axes
            const double a = hj[(c * 6 + 3) * N + i], b = hj[(c * 6 + 4) * N + i], e = hj[(c * 6 + 5) * N + i];
            worst = fmax(worst, fabs(sqrt(a * a + b * b + e * e) - 1.0));
        }
    printf("gripper_link at q = 0: (%.5f, %.5f, %.5f); max | |z_j| - 1 | over %lld configs: %.2e\n", x, y, z,
           (long long)N, worst);
    const int ok = fabs(x - 1.1281) < 1e-3 && fabs(y) < 1e-3 && fabs(z - 0.78601) < 1e-3 && worst < 1e-5;
    kin_plan_destroy(p);
    kin_model_destroy(m);
    kin_urdf_destroy(u);
    hipFree(dq);
    hipFree(dp);
    hipFree(dj);
    free(hq);
    free(hp);
    free(hj);
    printf(ok ? "OK\n" : "MISMATCH\n");
    return ok ? 0 : 2;
}
