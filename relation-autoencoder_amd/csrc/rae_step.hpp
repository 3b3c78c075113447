// Kernel argument block and exchange-record layout shared by the step kernels.
#pragma once
#include <stdint.h>

namespace rae {

// Per-example record in the exchange buffer (floats).  Layout is decoder-independent:
//   P (m) | dS (m) | V1 (r) | V2 (r) | dw1 (r) | dw2 (r) | coef (3*NJ) | loss (1) | pad
// SP       : V1 = wC1 = C1.P, V2 = wC2, dw1/dw2 = dCost/dwC1, dCost/dwC2,
//            coef[j] = (alpha_j, beta_j, gamma_j): record j's A-row gradient is
//            alpha_j*V1 + beta_j*V2 and its Ab gradient gamma_j.
// RESCAL / hybrid use the same slots with their own basis vectors (rae_bilinear.hpp).
struct RecLayout {
    int oP, odS, oV1, oV2, odw1, odw2, ocoef, oloss, rec;
    int oX, oY;   // bilinear factor vectors x_b, y_b (RESCAL/hybrid) ; 0 for SP
};

__host__ __device__ inline int align4(int x) { return (x + 3) & ~3; }

__host__ __device__ inline RecLayout make_layout(int dec, int m, int r, int s) {
    RecLayout L{};
    const int NJ = 2 + 2 * s;
    const int m4 = align4(m), r4 = align4(r);
    L.oP = 0;
    L.odS = m4;
    L.oV1 = 2 * m4;
    L.oV2 = L.oV1 + r4;
    L.odw1 = L.oV2 + r4;
    L.odw2 = L.odw1 + r4;
    int o = L.odw2 + r4;
    if (dec != 0) {          // bilinear factors + the two extra A-row basis vectors
        L.oX = o; o += r4;    // x_b  (left factor of dM_b)
        L.oY = o; o += r4;    // y_b  (right factor with a1)
    }
    L.ocoef = o;
    o += align4(3 * NJ);
    L.oloss = o;
    L.rec = align4(o + 1);
    return L;
}

struct StepArgs {
    // configuration
    int dec, opt;
    int64_t N, d, n;
    int m, r, s, l, L, rank;
    float lr, alpha, l1adj, l2adj, invD;
    int ext_reg, reg_on;
    // data
    const int32_t* indptr;
    const int32_t* indices;
    const float* values;
    const int32_t* args1;
    const int32_t* args2;
    const int32_t* neg1;
    const int32_t* neg2;
    int neg_mode;
    int64_t neg_stride;
    // parameters / accumulators
    float *W, *Wb, *A, *Ab, *C1, *C2, *R3;
    float *aW, *aWb, *aA, *aAb, *aC1, *aC2, *aR3;
    // exchange records
    float* ex;
    RecLayout lay;
    // row index of the global batches (rae_index.hpp), one slot per batch % index_window
    int HA, HW, RA, RW, posbits;
    int64_t index_window;
    int32_t *hdrA, *srecA, *urowA;      // urow*: interleaved (row, first position) pairs
    int32_t *hdrW, *srecW, *urowW;
    // batch addressing, outputs, scratch
    const int64_t* cursor;
    int64_t step_offset;
    float* costs;
    float* gWs;          // dense W gradient scratch (reg_on only)
    double* regpart;     // [nreg][2] L1/L2 partials of regularised rows
    int nregC;           // number of decoder-row partial slots
    int nregW;           // number of dense-W block partial slots
    float* base_cost;    // cost before the regulariser (reg_on only)
    int* err;            // device error word
    unsigned long long* stamps;   // diagnostic build only (RAE_STAMPS): phase timestamps
};

#ifdef RAE_STAMPS
#define RAE_STAMP(a, slot)                                                                  \
    do {                                                                                    \
        if ((a).stamps && threadIdx.x == 0)                                                 \
            (a).stamps[(size_t)blockIdx.x * 16 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define RAE_STAMP(a, slot) do { } while (0)
#endif

}  // namespace rae
