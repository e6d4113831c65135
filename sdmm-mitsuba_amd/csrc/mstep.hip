// mstep.hip -- stepwise blend, MAP M-step and component set-up on gfx950.
//
// Replaces (per EM iteration, all on the device, no host round trip):
//   stepwise blend      stepwise_tangent.h:685-743
//   MAP M-step          stepwise_tangent.h:745-980  (priors, exp of the mean in
//                       the old frame, PD test, stats re-centring)
//   normalisation/CDF   stepwise_tangent.h:992-1035, utils.h:64-102
//   MVTN::set           multivariate_tangent_normal.cpp:16-65 (+ conditioning
//                       mvtn.h:386-408, marginal mvtn.h:446-454)
// The M-step is O(K * 5^3): one thread per component, fp64 throughout (the
// "accurate" oracle mode), component parameters rounded to float at the end.
// FMA contraction is off so the fp64 op order equals oracle/sdmm_oracle.c's.
#include "sdmm_device.h"

#pragma clang fp contract(off)

namespace sdmm {

__device__ static void coordinates_d(const double n[3], double to[9]) {
    // Coordinates (utils.h:32-48)
    double sign = copysign(1.0, n[2]);
    const double a = -1.0 / (sign + n[2]);
    const double b = n[0] * n[1] * a;
    to[0] = 1.0 + sign * n[0] * n[0] * a; to[1] = sign * b; to[2] = -sign * n[0];
    to[3] = b; to[4] = sign + n[1] * n[1] * a; to[5] = -n[1];
    to[6] = n[0]; to[7] = n[1]; to[8] = n[2];
}

__device__ static double sinc_pi_d(double x) {
    // boost::math::sinc_pi
    const double taylor_0_bound = 2.220446049250313e-16;
    const double taylor_2_bound = sqrt(taylor_0_bound);
    const double taylor_n_bound = sqrt(taylor_2_bound);
    double ax = fabs(x);
    if (ax >= taylor_n_bound) return sin(x) / x;
    double result = 1.0;
    if (ax >= taylor_0_bound) {
        double x2 = x * x;
        result -= x2 / 6.0;
        if (ax >= taylor_2_bound) result += (x2 * x2) / 120.0;
    }
    return result;
}

// Eigen LLT<Lower>, unblocked (reads the lower triangle of row-major A).
template <int N>
__device__ static bool llt_d(const double* A, double* L) {
    for (int i = 0; i < N * N; ++i) L[i] = 0.0;
    for (int i = 0; i < N; ++i)
        for (int j = 0; j <= i; ++j) L[i * N + j] = A[i * N + j];
    for (int k = 0; k < N; ++k) {
        double x = L[k * N + k];
        for (int j = 0; j < k; ++j) x -= L[k * N + j] * L[k * N + j];
        if (!(x > 0.0)) return false;
        x = sqrt(x);
        L[k * N + k] = x;
        for (int i = k + 1; i < N; ++i) {
            double v = L[i * N + k];
            for (int j = 0; j < k; ++j) v -= L[i * N + j] * L[k * N + j];
            L[i * N + k] = v / x;
        }
    }
    return true;
}

template <int N>
__device__ static void tri_inv_d(const double* L, double* Li) {
    for (int i = 0; i < N * N; ++i) Li[i] = 0.0;
    for (int c = 0; c < N; ++c)
        for (int i = c; i < N; ++i) {
            double v = (i == c) ? 1.0 : 0.0;
            for (int j = c; j < i; ++j) v -= L[i * N + j] * Li[j * N + c];
            Li[i * N + c] = v / L[i * N + i];
        }
}

__device__ static void inv3_d(const double* m, double* r) {
    // Eigen compute_inverse_size3 (adjugate / det)
    double c00 = m[4] * m[8] - m[5] * m[7];
    double c10 = m[7] * m[2] - m[8] * m[1];
    double c20 = m[1] * m[5] - m[2] * m[4];
    double det = c00 * m[0] + c10 * m[3] + c20 * m[6];
    double invdet = 1.0 / det;
    r[0] = c00 * invdet; r[1] = c10 * invdet; r[2] = c20 * invdet;
    r[3] = (m[5] * m[6] - m[3] * m[8]) * invdet;
    r[4] = (m[8] * m[0] - m[6] * m[2]) * invdet;
    r[5] = (m[2] * m[3] - m[0] * m[5]) * invdet;
    r[6] = (m[3] * m[7] - m[4] * m[6]) * invdet;
    r[7] = (m[6] * m[1] - m[7] * m[0]) * invdet;
    r[8] = (m[0] * m[4] - m[1] * m[3]) * invdet;
}

// MVTN::set(mean, cov) in fp64, results rounded to float (oracle mode 1).
// have >= 0: the fp64 Cholesky of this cov was already attempted (the PD
// test's own, pd_test_keep) -- have = its success, Lk / Lik its L and L^-1 --
// and is not repeated (the same operations on the same doubles).
__device__ static void set_component(int k, const double* mean, const double* cov, const CanonDev& C,
                                     int have = -1, const double* Lk = nullptr, const double* Lik = nullptr) {
    float fm[6];
    for (int i = 0; i < 6; ++i) { fm[i] = (float)mean[i]; C.mean[6 * k + i] = fm[i]; }
    for (int i = 0; i < 25; ++i) C.cov[25 * k + i] = (float)cov[i];
    double md[3] = {(double)fm[3], (double)fm[4], (double)fm[5]};
    double tod[9];
    coordinates_d(md, tod);
    for (int i = 0; i < 9; ++i) C.to[9 * k + i] = (float)tod[i];
    double AA[9], AB[6], BA[6], BB[4], AAi[9], P[6], S[4];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) AA[3 * i + j] = cov[5 * i + j];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 2; ++j) AB[2 * i + j] = cov[5 * i + 3 + j];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j) BA[3 * i + j] = cov[5 * (3 + i) + j];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) BB[2 * i + j] = cov[5 * (3 + i) + 3 + j];
    inv3_d(AA, AAi);
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j) {
            double v = 0.0;
            for (int l = 0; l < 3; ++l) v += BA[3 * i + l] * AAi[3 * l + j];
            P[3 * i + j] = v;
        }
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) {
            double v = 0.0;
            for (int l = 0; l < 3; ++l) v += P[3 * i + l] * AB[2 * l + j];
            S[2 * i + j] = BB[2 * i + j] - v;
        }
    for (int i = 0; i < 6; ++i) C.muPremult[6 * k + i] = (float)P[i];
    for (int i = 0; i < 4; ++i) C.condCov[4 * k + i] = (float)S[i];
    double Lb[25], Lib[25];
    const double* L = Lk;
    const double* Li = Lik;
    int ok = 1;
    bool chol;
    if (have < 0) {
        chol = llt_d<5>(cov, Lb);
        if (chol) tri_inv_d<5>(Lb, Lib);
        L = Lb;
        Li = Lib;
    } else {
        chol = have != 0;
    }
    if (chol) {
        double det = 1.0;
        for (int i = 0; i < 5; ++i) det *= L[6 * i];
        for (int i = 0; i < 25; ++i) {
            C.cholL[25 * k + i] = (float)L[i];
            C.cholLInv[25 * k + i] = (float)Li[i];
        }
        C.detInv[k] = (float)(1.0 / det);
    } else {
        ok = 0;
    }
    double A3[9], L3[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) A3[3 * i + j] = cov[5 * i + j];
    if (llt_d<3>(A3, L3)) {
        for (int i = 0; i < 9; ++i) C.margL[9 * k + i] = (float)L3[i];
        C.margDetInv[k] = (float)(1.0 / (L3[0] * L3[4] * L3[8]));
    }
    double L2[4];
    if (llt_d<2>(S, L2)) {
        double det2 = L2[0] * L2[3];
        C.condL[4 * k + 0] = (float)L2[0]; C.condL[4 * k + 1] = 0.0f;
        C.condL[4 * k + 2] = (float)L2[2]; C.condL[4 * k + 3] = (float)L2[3];
        C.condLInv[4 * k + 0] = (float)(L2[3] / det2);
        C.condLInv[4 * k + 1] = 0.0f;
        C.condLInv[4 * k + 2] = (float)(-L2[2] / det2);
        C.condLInv[4 * k + 3] = (float)(L2[0] / det2);
        C.condDetInv[k] = (float)(1.0 / det2);
    }
    C.valid[k] = ok;
}

// Packed E-step and guide records of component k (k < Kp; k >= K is padding).
// weights == false: every field but the weight ones (EP_PI, EP_DIPI, GP_W:
// mstep_spread_kernel's finish writes them once the weights are final).
__device__ static void pack_component(int k, int K, int Kp, const CanonDev& C, float* ep, float* gp,
                                      float norm5, bool weights = true) {
    float e[EP_FIELDS];
    float g[GP_FIELDS];
    for (int f = 0; f < EP_FIELDS; ++f) e[f] = 0.0f;
    for (int f = 0; f < GP_FIELDS; ++f) g[f] = 0.0f;
    if (k < K) {
        const float w = C.weights[k];
        const float* mu = C.mean + 6 * k;
        const float* Li = C.cholLInv + 25 * k;
        const float* to = C.to + 9 * k;
        e[EP_MU0] = mu[0]; e[EP_MU1] = mu[1]; e[EP_MU2] = mu[2];
        const int lidx[15] = {0, 5, 6, 10, 11, 12, 15, 16, 17, 18, 20, 21, 22, 23, 24};
        for (int i = 0; i < 15; ++i) e[EP_L00 + i] = Li[lidx[i]];
        for (int i = 0; i < 9; ++i) e[EP_R00 + i] = to[i];
        e[EP_DI] = C.detInv[k];
        e[EP_PI] = C.valid[k] ? w : 0.0f;
        for (int i = 0; i < 3; ++i) {
            e[EP_A0 + i] = Li[18] * to[i];
            e[EP_B0 + i] = Li[23] * to[i] + Li[24] * to[3 + i];
        }
        e[EP_DIPI] = e[EP_DI] * e[EP_PI];
        for (int m = 0; m < 5; ++m) {
            const int row = m * (m + 1) / 2;          // packed lower-triangle row of L^-1
            const int jn = m < 3 ? m + 1 : 3;
            double acc = 0.0;
            for (int j = 0; j < jn; ++j)
                acc += (double)e[EP_L00 + row + j] * ((double)mu[j] - (double)kOrigin);
            e[EP_NC0 + m] = (float)(-acc);
        }
        {
            const double n2 = (double)to[6] * (double)to[6] + (double)to[7] * (double)to[7] +
                              (double)to[8] * (double)to[8];
            e[EP_CN] = (float)(0.5 * (1.0 - n2));
        }
        g[GP_W] = w;
        g[GP_MU0] = mu[0]; g[GP_MU1] = mu[1]; g[GP_MU2] = mu[2];
        const float* ML = C.margL + 9 * k;
        g[GP_ML00] = ML[0]; g[GP_ML10] = ML[3]; g[GP_ML11] = ML[4];
        g[GP_ML20] = ML[6]; g[GP_ML21] = ML[7]; g[GP_ML22] = ML[8];
        g[GP_MDI] = C.margDetInv[k];
        for (int i = 0; i < 6; ++i) g[GP_P00 + i] = C.muPremult[6 * k + i];
        for (int i = 0; i < 9; ++i) g[GP_T00 + i] = to[i];
        g[GP_CL00] = C.condL[4 * k + 0]; g[GP_CL10] = C.condL[4 * k + 2]; g[GP_CL11] = C.condL[4 * k + 3];
        for (int i = 0; i < 4; ++i) g[GP_CI00 + i] = C.condLInv[4 * k + i];
        g[GP_CDI] = C.condDetInv[k];
        const int rml[3] = {GP_RML00, GP_RML11, GP_RML22};
        const float mld[3] = {g[GP_ML00], g[GP_ML11], g[GP_ML22]};
        for (int i = 0; i < 3; ++i) {
            const uint64_t bits = __builtin_bit_cast(uint64_t, 1.0 / (double)mld[i]);
            g[rml[i]] = __builtin_bit_cast(float, (uint32_t)bits);
            g[rml[i] + 1] = __builtin_bit_cast(float, (uint32_t)(bits >> 32));
        }
    }
    for (int f = 0; f < EP_FIELDS; ++f)
        if (weights || (f != EP_PI && f != EP_DIPI)) ep[f * Kp + k] = e[f];
    for (int f = 0; f < GP_FIELDS; ++f)
        if (weights || f != GP_W) gp[k * GP_STRIDE + f] = g[f];
}

// createCdf(false) then configure()'s createCdf(true) (float, sequential);
// executed by one thread.
__device__ static void weights_cdf(float* w, float* cdf, int K, bool first_partial) {
    if (first_partial) {
        float acc = 0.0f;
        for (int k = 0; k < K; ++k) { acc += w[k]; cdf[k] = acc; }
    }
    float sum = 0.0f;
    for (int k = 0; k < K; ++k) sum += w[k];
    if (sum == 0.0f) return;
    for (int k = 0; k < K; ++k) w[k] = w[k] / sum;
    float acc = 0.0f;
    for (int k = 0; k < K; ++k) { acc += w[k]; cdf[k] = acc; }
}

// ---------------------------------------------------------------------------
// set() for all components from (mean, cov) given in fp64, then configure().
__global__ void __launch_bounds__(512)
set_all_kernel(int K, int Kp, const double* __restrict__ mean, const double* __restrict__ cov,
               CanonDev C, float* ep, float* gp, float norm5) {
    const int k = threadIdx.x;
    if (k < K) set_component(k, mean + 6 * k, cov + 25 * k, C);
    __syncthreads();
    if (k == 0) weights_cdf(C.weights, C.cdf, K, false);
    __syncthreads();
    for (int kk = k; kk < Kp; kk += blockDim.x) pack_component(kk, K, Kp, C, ep, gp, norm5);
}

// Re-derive the packed records only (after sdmm_set_params of weights).
__global__ void __launch_bounds__(512)
pack_all_kernel(int K, int Kp, CanonDev C, float* ep, float* gp, float norm5) {
    for (int kk = threadIdx.x; kk < Kp; kk += blockDim.x) pack_component(kk, K, Kp, C, ep, gp, norm5);
}

// ---------------------------------------------------------------------------
// jmm::isPositiveDefinite (opt/util.h:29-41): all eigenvalues of the symmetric
// matrix read from the lower triangle (SelfAdjointEigenSolver) are > 0.  Cyclic
// Jacobi in fp64, operation for operation the oracle's is_pd_f64
// (oracle/sdmm_oracle.c), so GPU and oracle kill the same components -- a
// Cholesky success test differs from the eigenvalue test for near-singular
// covariances.
__device__ static bool pd_jacobi_d(const double* A) {
    constexpr int n = 5;
    double a[25];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) a[i * n + j] = (i >= j) ? A[i * n + j] : A[j * n + i];
    for (int i = 0; i < n * n; ++i)
        if (!isfinite(a[i])) return false;
    for (int sweep = 0; sweep < 64; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) off += a[p * n + q] * a[p * n + q];
        if (off == 0.0) break;
        for (int p = 0; p < n; ++p) {
            for (int q = p + 1; q < n; ++q) {
                const double apq = a[p * n + q];
                if (apq == 0.0) continue;
                const double app = a[p * n + p], aqq = a[q * n + q];
                const double theta = (aqq - app) / (2.0 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                if (!isfinite(theta * theta)) t = 1.0 / (2.0 * theta);
                const double cs = 1.0 / sqrt(t * t + 1.0), sn = t * cs;
                for (int k = 0; k < n; ++k) {
                    const double akp = a[k * n + p], akq = a[k * n + q];
                    a[k * n + p] = cs * akp - sn * akq;
                    a[k * n + q] = sn * akp + cs * akq;
                }
                for (int k = 0; k < n; ++k) {
                    const double apk = a[p * n + k], aqk = a[q * n + k];
                    a[p * n + k] = cs * apk - sn * aqk;
                    a[q * n + k] = sn * apk + cs * aqk;
                }
            }
        }
    }
    for (int i = 0; i < n; ++i)
        if (!(a[i * n + i] > 0.0)) return false;
    return true;
}

// The kill test with a fast accept: the fp64 Cholesky A + E = L L^T (|E| ~ 5e-16
// |A|) with lambda_min(A + E) >= 1 / |L^-1|_F^2 (|A^-1|_2 <= |L^-T|_F |L^-1|_F).
// When that lower bound exceeds 1e-9 |A|_F, lambda_min(A) is positive by six
// orders of magnitude more than Jacobi's own rounding (~n eps |A|), so Jacobi
// would report positive definite too; every other case (a failed or
// near-singular factorisation) runs the Jacobi test itself.  Same decisions as
// pd_jacobi_d alone, at the cost of a Cholesky for the common component.
__device__ static bool pd_test_keep(const double* A, double* L, double* Li, bool* have) {
    *have = llt_d<5>(A, L);
    if (*have) {
        tri_inv_d<5>(L, Li);
        double fro = 0.0, an = 0.0;
        for (int i = 0; i < 25; ++i) {
            fro += Li[i] * Li[i];
            const int r = i / 5, c = i % 5;
            const double a = (r >= c) ? A[i] : A[5 * c + r];   // the lower triangle, mirrored
            an += a * a;
        }
        if (isfinite(fro) && 1.0 / fro > 1e-9 * sqrt(an)) return true;
    }
    return pd_jacobi_d(A);
}
__device__ static bool pd_test_d(const double* A) {
    double L[25], Li[25];
    bool have;
    return pd_test_keep(A, L, Li, &have);
}

// ---------------------------------------------------------------------------
// One stepwise M-step from the compact fp64 stats [H, wsum, W, M, Clow], in
// four phases so that it can run as one workgroup (the batched per-leaf
// M-step: a workgroup per leaf) or spread over the chip (a single mixture:
// phase 2 and the packing over K threads of many workgroups).  The phases are
// the same code either way, so both forms give the same bits.
//   1. scalars   blend of the totals, eta, the prior factors -> sh[8]
//   2. component the blend, MAP update, PD test, stats re-centring of component
//                k; the accepted (mean, cov) go to wmean/wcov, setk[k] = 1;
//                then MVTN::set of the accepted components (a separate pass:
//                the fp64 footprints of the two never overlap)
//   3. finish    weights normalised over the components, CDF, iterations + 1
//   4. pack      the E-step / guide records of every component
// sh: [status, eta, weightSum, 1/hTW, invGlobal, invMix]; status 0: weightSum
// == 0, optimize() returns early (nothing changes).
// sh as above; upd: the blended [heuristicTotalWeight, sgH, normalization]
// the scalars take (written by mstep_scalars_store, after every reader).
__device__ __forceinline__ void mstep_scalars_compute(const double* __restrict__ stats, int64_t nSamples, int K,
                                                      const EmStateDev& S, double* sh, double* upd) {
    if (nSamples < 0) nSamples = (int64_t)stats[2 + ST_FIELDS * K];   // sharded: the all-reduced count
    const double weightSum = stats[1];
    sh[0] = (weightSum == 0.0) ? 0.0 : 1.0;
    if (weightSum != 0.0) {
        const int it = (int)S.scalars[SC_IT];
        const double alpha = S.scalars[SC_ALPHA];
        const double learningRate = (double)0.2f;
        const double eta = pow(learningRate * (double)it + 1.0, -alpha);
        double hTW = S.scalars[SC_HTW];
        hTW *= (1.0 - eta);
        hTW += eta * weightSum;
        upd[0] = hTW;
        double gH = S.scalars[SC_SGH] * (1.0 - eta);
        gH = eta * stats[0] + gH;
        upd[1] = gH;
        const double norm = (double)(float)S.scalars[SC_NORM];
        upd[2] = (double)(float)((1.0 - eta) * norm + eta * weightSum / (double)nSamples);
        const int cutoff = (int)S.scalars[SC_CUT];
        const int cut = (cutoff < it) ? cutoff : it;
        // 3^cut and 2^cut are exact in fp64 for cut <= 33 (the trainingCutoff
        // is 32), so the products equal any correctly rounded pow (the
        // oracle's libm pow); a serial fp64 pow was ~2 us each of the M-step
        double p3 = 1.0;
        for (int i = 0; i < cut && cut <= 33; ++i) p3 *= 3.0;
        if (cut > 33) p3 = pow(3.0, (double)cut);
        const double invGlobal = 1.0 / p3;
        const double invMix = 1.0 / ldexp(1.0, cut);
        sh[1] = eta;
        sh[2] = weightSum;
        sh[3] = 1.0 / hTW;
        sh[4] = invGlobal;
        sh[5] = invMix;
    }
}
__device__ __forceinline__ void mstep_scalars_store(const EmStateDev& S, const double* sh, const double* upd) {
    if (sh[0] != 0.0) {
        S.scalars[SC_HTW] = upd[0];
        S.scalars[SC_SGH] = upd[1];
        S.scalars[SC_NORM] = upd[2];
    }
    S.scalars[SC_STATUS] = sh[0];
}
__device__ __forceinline__ void mstep_scalars(const double* __restrict__ stats, int64_t nSamples, int K,
                                              const EmStateDev& S, double* sh) {
    double upd[3];
    mstep_scalars_compute(stats, nSamples, K, S, sh, upd);
    mstep_scalars_store(S, sh, upd);
}

// Component k's inputs to the M-step (its stats, stepwise state, priors,
// weight and frame), loaded ahead of the scalars so that the loads overlap
// them (mstep_spread_kernel).
struct CompIn {
    double st[ST_FIELDS];   // W, M0..M4, Clow (the compact order)
    double T, sgW, sgM[5], sgC[25], ni;
    float bP[25], bD[9], to[9], w, di;
    int valid;
    bool decp;
};
__device__ __forceinline__ void load_comp_in(int k, int K, const double* __restrict__ stats, const CanonDev& C,
                                             const EmStateDev& S, CompIn& in) {
    in.st[0] = stats[2 + k];
    for (int i = 0; i < 5; ++i) in.st[1 + i] = stats[2 + K + 5 * k + i];
    for (int i = 0; i < 15; ++i) in.st[6 + i] = stats[2 + 6 * K + 15 * k + i];
    in.T = S.T[k];
    in.sgW = S.sgW[k];
    for (int i = 0; i < 5; ++i) in.sgM[i] = S.sgM[5 * k + i];
    for (int i = 0; i < 25; ++i) in.sgC[i] = S.sgC[25 * k + i];
    in.ni = S.scalars[SC_NI];
    in.decp = S.scalars[SC_DECP] != 0.0;
    for (int i = 0; i < 25; ++i) in.bP[i] = S.bPriors[25 * k + i];
    for (int i = 0; i < 9; ++i) in.bD[i] = S.bDepth[9 * k + i];
    for (int i = 0; i < 9; ++i) in.to[i] = C.to[9 * k + i];
    in.w = C.weights[k];
    in.di = C.detInv[k];
    in.valid = C.valid[k];
}

// wm, wc: component k's accepted (mean, cov) slots; L5 / Li5 / have (or
// nullptr): keep the PD test's fp64 factorisation for set_component.
__device__ __forceinline__ void mstep_component(int k, int K, const CompIn& in, const EmStateDev& S,
                                                const double* sh, double* newW, int* setk,
                                                double* __restrict__ wm, double* __restrict__ wc,
                                                double* L5 = nullptr, double* Li5 = nullptr, bool* have = nullptr) {
    const double eta = sh[1], weightSum = sh[2], invTotalWeight = sh[3];
    const double invGlobal = sh[4], invMix = sh[5];
    const double ni = in.ni;
    const bool decreasePrior = in.decp;
    setk[k] = 0;
    double T = in.T;
    T *= (1.0 - eta);
    T += eta * weightSum;
    S.T[k] = T;
    // statsGlobal *= (1 - eta); stats.sumProductInto(statsGlobal, eta)
    const double oneMinus = 1.0 - eta;
    double gW = in.sgW * oneMinus;
    gW = eta * in.st[0] + gW;
    double gM[5], gC[25];
    for (int i = 0; i < 5; ++i) {
        double v = in.sgM[i] * oneMinus;
        gM[i] = eta * in.st[1 + i] + v;
    }
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j) {
            const int a = i > j ? i : j, b = i > j ? j : i;
            const double sc = in.st[6 + a * (a + 1) / 2 + b];
            double v = in.sgC[5 * i + j] * oneMinus;
            gC[5 * i + j] = eta * sc + v;
        }
    // statsGlobalNormalized
    const double nW = gW * invTotalWeight;
    double nM[5], nC[25];
    for (int i = 0; i < 5; ++i) nM[i] = gM[i] * invTotalWeight;
    for (int i = 0; i < 25; ++i) nC[i] = gC[i] * invTotalWeight;

    double decNi = ni;
    double decA = 100.0 / (double)K;
    double decB[25];
    for (int i = 0; i < 25; ++i) decB[i] = decA * (double)in.bP[i];
    if (decreasePrior) {
        for (int i = 0; i < 25; ++i) decB[i] = decB[i] * invMix;
        decA = decA * invMix;
        decNi = ni * invGlobal;
    }
    const double invW = 1.0 / nW;
    const double invMatNorm = 1.0 / (0.05 * decA + nW);
    double w_new;
    if (in.w == 0.0f) {
        w_new = 0.0;                       // dead stays dead (:785)
    } else if (!isfinite(invW)) {
        w_new = decNi + nW;                // weak component (:791)
    } else {
        w_new = decNi + nW;
        double mean5[5], cov[25];
        for (int i = 0; i < 5; ++i) mean5[i] = nM[i] * invW;
        for (int i = 0; i < 5; ++i)
            for (int j = 0; j < 5; ++j) cov[5 * i + j] = nC[5 * i + j] - nM[i] * mean5[j];
        for (int i = 0; i < 25; ++i) cov[i] += decB[i];
        for (int i = 0; i < 25; ++i) cov[i] *= invMatNorm;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) cov[5 * i + j] += (double)in.bD[3 * i + j];
        // exp of the new tangent mean in the OLD frame (:845-852)
        double to[9], emb[6];
        for (int i = 0; i < 9; ++i) to[i] = (double)in.to[i];
        {
            const double t0 = mean5[3], t1 = mean5[4];
            const double length = sqrt(t0 * t0 + t1 * t1);
            if (length >= kPi) {
                for (int i = 0; i < 6; ++i) emb[i] = 0.0;
            } else {
                const double sc = sinc_pi_d(length);
                const double rel0 = t0 * sc, rel1 = t1 * sc, rel2 = cos(length);
                emb[0] = mean5[0]; emb[1] = mean5[1]; emb[2] = mean5[2];
                emb[3] = to[0] * rel0 + to[3] * rel1 + to[6] * rel2;
                emb[4] = to[1] * rel0 + to[4] * rel1 + to[7] * rel2;
                emb[5] = to[2] * rel0 + to[5] * rel1 + to[8] * rel2;
            }
        }
        if (!(L5 ? pd_test_keep(cov, L5, Li5, have) : pd_test_d(cov))) {
            w_new = 0.0;                   // not positive definite: kill (:945-960)
        } else {
            for (int i = 0; i < 6; ++i) wm[i] = emb[i];
            for (int i = 0; i < 25; ++i) wc[i] = cov[i];
            setk[k] = 1;
            for (int i = 0; i < 5; ++i)
                for (int j = 0; j < 5; ++j) nC[5 * i + j] -= nM[i] * mean5[j];
            const double condStat[5] = {nM[0], nM[1], nM[2], 0.0, 0.0};
            const double condNew[5] = {mean5[0], mean5[1], mean5[2], 0.0, 0.0};
            for (int i = 0; i < 5; ++i)
                for (int j = 0; j < 5; ++j) nC[5 * i + j] += condStat[i] * condNew[j];
            for (int i = 0; i < 25; ++i) gC[i] = nC[i] * T;
            gM[3] = 0.0;
            gM[4] = 0.0;
        }
    }
    newW[k] = w_new;
    S.sgW[k] = gW;
    for (int i = 0; i < 5; ++i) S.sgM[5 * k + i] = gM[i];
    for (int i = 0; i < 25; ++i) S.sgC[25 * k + i] = gC[i];
}

// The finish: the three order-dependent sums (the fp64 total of newW, the
// float prefix of the weights -- whose last value is also their float total
// --, the float prefix of the normalised weights) are each ONE thread's
// sequential chain over LDS (loads batched ahead of the adds), the
// elementwise divisions and roundings run on every thread (t of nt) between
// them; sync() orders the LDS traffic (a workgroup barrier, or within one
// wave).  The readlane chains before took ~16 us of a K = 128 M-step
// (tools/em_phases.py with SDMM_MSTEP_STOP builds).
// newW, wl, cl: LDS, K doubles / floats; sh2: 2 doubles of LDS.
template <class Sync>
__device__ __forceinline__ void mstep_finish(int K, const EmStateDev& S, const double* newW, float* wl, float* cl,
                                             double* sh2, int t, int nt, Sync sync) {
    if (t == 0) {
        double sum = 0.0;
        int k = 0;
        for (; k + 8 <= K; k += 8) {
            double v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = newW[k + i];
#pragma unroll
            for (int i = 0; i < 8; ++i) sum += v[i];
        }
        for (; k < K; ++k) sum += newW[k];
        sh2[0] = sum;
    }
    sync();
    const double sum = sh2[0];
    for (int k = t; k < K; k += nt) {
        double nw = newW[k];
        if (sum != 0.0) nw = nw / sum;
        wl[k] = (float)nw;
    }
    sync();
    // createCdf(false): the unnormalised prefix (kept if the total is 0); its
    // last value is the float total fs
    auto prefix = [&]() {
        float acc = 0.0f;
        int k = 0;
        for (; k + 8 <= K; k += 8) {
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = wl[k + i];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                acc += v[i];
                cl[k + i] = acc;
            }
        }
        for (; k < K; ++k) {
            acc += wl[k];
            cl[k] = acc;
        }
        return acc;
    };
    if (t == 0) sh2[1] = (double)prefix();
    sync();
    const float fs = (float)sh2[1];
    if (fs != 0.0f) {
        for (int k = t; k < K; k += nt) wl[k] = wl[k] / fs;
        sync();
        if (t == 0) (void)prefix();
    }
    if (t == 0) S.scalars[SC_IT] = S.scalars[SC_IT] + 1.0;
}
__device__ __forceinline__ void mstep_finish_block(int K, const EmStateDev& S, const double* newW, float* wl,
                                                   float* cl, double* sh2) {
    mstep_finish(K, S, newW, wl, cl, sh2, (int)threadIdx.x, (int)blockDim.x, [] { __syncthreads(); });
}

// The four phases in one workgroup (the batched per-leaf M-step).
__device__ __forceinline__ void mstep_body(int K, int Kp, const double* __restrict__ stats, int64_t nSamples,
                                           CanonDev C, EmStateDev S, float* ep, float* gp, float norm5,
                                           double* __restrict__ wmean, double* __restrict__ wcov) {
    __shared__ double sh[8];
    __shared__ double sh2[2];
    extern __shared__ double newW[];
    int* setk = (int*)(newW + K);
    const int t = threadIdx.x;
// SDMM_MSTEP_STOP=n (diagnostic builds, tools/build_variant.sh): return after
// phase n, for a phase breakdown by subtraction (not results)
#ifndef SDMM_MSTEP_STOP
#define SDMM_MSTEP_STOP 99
#endif
    if (t == 0) mstep_scalars(stats, nSamples, K, S, sh);
    __syncthreads();
    if (sh[0] == 0.0 || SDMM_MSTEP_STOP <= 1) return;  // optimize() returns early when weightSum == 0
    for (int k = t; k < K; k += blockDim.x) {
        CompIn in;
        load_comp_in(k, K, stats, C, S, in);
        mstep_component(k, K, in, S, sh, newW, setk, wmean + 6 * k, wcov + 25 * k);
    }
    __syncthreads();
    if (SDMM_MSTEP_STOP <= 2) return;
    for (int k = t; k < K; k += blockDim.x)
        if (setk[k]) set_component(k, wmean + 6 * k, wcov + 25 * k, C);
    __syncthreads();
    if (SDMM_MSTEP_STOP <= 3) return;
    // dynamic LDS: newW (8K bytes), setk (4K) -- reused as wl --, cl (4K)
    float* wl = (float*)setk;
    float* cl = wl + K;
    mstep_finish_block(K, S, newW, wl, cl, sh2);
    __syncthreads();
    if (SDMM_MSTEP_STOP <= 4) return;
    for (int k = t; k < K; k += blockDim.x) {
        C.weights[k] = wl[k];
        C.cdf[k] = cl[k];
    }
    __syncthreads();
    for (int kk = t; kk < Kp; kk += blockDim.x) pack_component(kk, K, Kp, C, ep, gp, norm5);
}

// Batched M-step: workgroup b updates mixture b of the table (per-leaf EM).
__global__ void __launch_bounds__(512)
mstep_batched_kernel(int K, int Kp, const MixDesc* __restrict__ mixes, float norm5) {
    const MixDesc& d = mixes[blockIdx.x];
    const int64_t n = d.ncount ? (int64_t)*d.ncount : d.n;
    if (n <= 0) return;   // no samples: optimize() returns early (weightSum == 0)
    mstep_body(K, Kp, d.stats, n, d.C, d.S, d.ep, d.gp, norm5, d.wmean, d.wcov);
}

// The single-mixture M-step spread over ceil(Kp / 64) workgroups of two
// waves (round 4: one workgroup, 20 us at K = 128 -- a latency chain per
// component, with 88 VGPRs spilled at its 512-thread bound).  Wave 0 of
// workgroup b owns components 64 b + lane: the blend / MAP / PD test, then
// MVTN::set from the PD test's own fp64 factorisation and every record field
// but the weight ones, all in one thread (nothing goes through memory).  The
// workgroup whose blends complete last (device-scope counter count[0],
// wrapped back to 0 by that arrival's atomicInc) runs the order-dependent
// finish on its wave 1 while its wave 0 sets: the weights normalised, both CDF
// prefixes, the scalars, and every record's weight fields -- from the valid
// flag and detInv each blend publishes beside its weight (what its set will
// leave).  The
// operations are mstep_body's, so the results are bitwise those of the
// batched per-leaf form.
__global__ void __launch_bounds__(128)
mstep_spread_kernel(int K, int Kp, const double* __restrict__ stats, int64_t nSamples, CanonDev C, EmStateDev S,
                    float* ep, float* gp, float norm5, double* scratch, unsigned* count) {
    // scratch: newW (K doubles), the valid flags and detInv after the set
    double* newW = scratch;
    float* dinew = (float*)(scratch + K);
    int* vnew = (int*)(scratch + 2 * K);
    __shared__ double sh[8];
    __shared__ double upd[3];
    __shared__ double sh2[2];
    __shared__ double nwl[512];
    __shared__ float wl[512], cl[512];
    __shared__ int role;   // bit 0: this workgroup runs the finish
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const unsigned nb = gridDim.x;
    const int k = (int)blockIdx.x * 64 + lane;
    // wave 1 forms the scalars while wave 0 loads its components' inputs
    CompIn in;
    if (wv == 0 && k < K) load_comp_in(k, K, stats, C, S, in);
    if (t == 64) mstep_scalars_compute(stats, nSamples, K, S, sh, upd);
    __syncthreads();
    if (sh[0] == 0.0) {   // optimize() returns early when weightSum == 0
        if (blockIdx.x == 0 && t == 0) S.scalars[SC_STATUS] = 0.0;
        return;
    }
    // SDMM_MSTEP_STOP=n (diagnostic builds): return after stage n -- 1 the
    // loads + scalars, 2 the blends, 3 the first counter, 4 set / finish,
    // 5 the records -- for a breakdown by subtraction (not results)
    if (SDMM_MSTEP_STOP <= 1) return;
    __shared__ int setk[512];
    double emb[6], cov[25], L[25], Li[25];
    bool have = false;
    if (wv == 0) {
        if (k < K) {
            mstep_component(k, K, in, S, sh, newW, setk, emb, cov, L, Li, &have);
            // the valid flag and detInv the set below leaves (set_component:
            // 1 / det of the Cholesky when it succeeds, else unchanged), so
            // that the finish can form the weight fields without waiting
            int v = in.valid;
            float di = in.di;
            if (setk[k]) {
                v = have ? 1 : 0;
                if (have) {
                    double det = 1.0;
                    for (int i = 0; i < 5; ++i) det *= L[6 * i];
                    di = (float)(1.0 / det);
                }
            }
            vnew[k] = v;
            dinew[k] = di;
        }
        if (SDMM_MSTEP_STOP <= 2) return;
        __threadfence();
        // atomicInc wraps to 0 on the last arrival: the counter is re-armed by
        // the same atomic that elects the finish, so no launch depends on a
        // later store of an earlier one (an aborted launch cannot leave it set)
        if (lane == 0) role = (atomicInc(&count[0], nb - 1) == nb - 1) ? 1 : 0;
    }
    if (SDMM_MSTEP_STOP <= 2) return;
    __syncthreads();
    if (SDMM_MSTEP_STOP <= 3) return;
    if (wv == 0) {
        if (k < K && setk[k]) set_component(k, emb, cov, C, have ? 1 : 0, L, Li);
        if (SDMM_MSTEP_STOP <= 4) return;
        if (k < Kp) pack_component(k, K, Kp, C, ep, gp, norm5, false);
        if (SDMM_MSTEP_STOP <= 5) return;
    } else {
        if (!role) return;
        __threadfence();
        for (int i = lane; i < K; i += 64) nwl[i] = newW[i];
        auto wave_sync = [] {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __builtin_amdgcn_wave_barrier();
        };
        wave_sync();
        mstep_finish(K, S, nwl, wl, cl, sh2, lane, 64, wave_sync);
        if (SDMM_MSTEP_STOP <= 4) return;
        wave_sync();
        for (int i = lane; i < K; i += 64) {
            C.weights[i] = wl[i];
            C.cdf[i] = cl[i];
        }
        if (lane == 0) mstep_scalars_store(S, sh, upd);
        if (SDMM_MSTEP_STOP <= 5) return;
        // every record's weight fields (pack_component's, from the valid
        // flags and detInv the blends published)
        for (int i = lane; i < Kp; i += 64) {
            float pi = 0.0f, dipi = 0.0f, w = 0.0f;
            if (i < K) {
                w = wl[i];
                pi = vnew[i] ? w : 0.0f;
                dipi = dinew[i] * pi;
            }
            ep[EP_PI * Kp + i] = pi;
            ep[EP_DIPI * Kp + i] = dipi;
            gp[i * GP_STRIDE + GP_W] = w;
        }
    }
}

__global__ void set_f64_kernel(double* p, double v) { *p = v; }

// StepwiseTangentEM constructor state: scalars, diagonal bPriors (bprior[i])
// and bDepth (eps) per component
struct InitScalars {
    double v[SC_COUNT];
    float bprior[5];
};
__global__ void init_state_kernel(int K, InitScalars a, float eps, double* __restrict__ sc, float* __restrict__ bp,
                                  float* __restrict__ bd) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k == 0)
        for (int i = 0; i < SC_COUNT; ++i) sc[i] = a.v[i];
    if (k >= K) return;
    for (int i = 0; i < 25; ++i) bp[25 * k + i] = (i % 6 == 0) ? a.bprior[i / 6] : 0.0f;
    for (int i = 0; i < 9; ++i) bd[9 * k + i] = (i % 4 == 0) ? eps : 0.0f;
}

// Batched initialisation: mixture b takes its weights (K f32), means (6K f32),
// covs (25K f32), bPriors (25K f32), bDepth (9K f32) from a device staging
// block and runs set_all (MVTN::set per component on the fp64-widened mean
// and covariance, CDF, packing).
struct InitDesc {
    CanonDev C;
    float *ep, *gp, *bp, *bd;
    double *tmean, *tcov;
};
__global__ void __launch_bounds__(512)
set_all_batched_kernel(int K, int Kp, const InitDesc* __restrict__ tab, const char* __restrict__ staging, size_t per,
                       float norm5) {
    const InitDesc d = tab[blockIdx.x];
    const char* b = staging + per * (size_t)blockIdx.x;
    const float* w = (const float*)b;
    const float* mean = (const float*)(b + 4 * (size_t)K);
    const float* cov = (const float*)(b + 28 * (size_t)K);
    const float* bp = (const float*)(b + 128 * (size_t)K);
    const float* bd = (const float*)(b + 228 * (size_t)K);
    const int t = threadIdx.x;
    for (int i = t; i < K; i += blockDim.x) d.C.weights[i] = w[i];
    for (int i = t; i < 25 * K; i += blockDim.x) d.bp[i] = bp[i];
    for (int i = t; i < 9 * K; i += blockDim.x) d.bd[i] = bd[i];
    __syncthreads();
    for (int k = t; k < K; k += blockDim.x) {
        double m[6], c[25];
        for (int i = 0; i < 6; ++i) m[i] = (double)mean[6 * k + i];
        for (int i = 0; i < 25; ++i) c[i] = (double)cov[25 * k + i];
        set_component(k, m, c, d.C);
    }
    __syncthreads();
    if (t == 0) weights_cdf(d.C.weights, d.C.cdf, K, false);
    __syncthreads();
    for (int kk = t; kk < Kp; kk += blockDim.x) pack_component(kk, K, Kp, d.C, d.ep, d.gp, norm5);
}

// uniformHemisphereInit (mixture_model_init.h:79-242, the kMeansPlusPlus ==
// false branch; :130-138 the k-means++ draws skipped) on the device: mixture
// b's staging block, in the layout set_all_batched_kernel reads, from its npos
// positions / normals, spatial distance and PCG32 seed.  The host version
// (sdmm_api.cpp hemisphere_init) wrote ~35 KB per K = 128 mixture into pinned
// memory for an upload; here only the inputs travel.  Same float and double
// operations in the same order (contraction off; the float square root taken
// through the correctly rounded double one, as the host's std::sqrt(float)
// rounds), so the results are the host's bit for bit except where the
// device's double cos / sin and the host libm's round to different floats.
struct HemiGenArgs {
    const float* pos;      // [n][npos][3]
    const float* nrm;      // [n][npos][3]
    const float* dist;     // [n] minimum spatial distance
    const uint64_t* seed;  // [n]
    int skip;              // draws already taken from each stream
    float depth_prior;
};
struct Pcg32Dev {
    uint64_t state, inc;
    __device__ void seed(uint64_t initstate, uint64_t initseq) {
        state = 0u;
        inc = (initseq << 1u) | 1u;
        next_uint();
        state += initstate;
        next_uint();
    }
    __device__ uint32_t next_uint() {
        const uint64_t old = state;
        state = old * 0x5851f42d4c957f2dULL + inc;
        const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        const uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((~rot + 1u) & 31));
    }
    __device__ float next_float() {
        return __builtin_bit_cast(float, (next_uint() >> 9) | 0x3f800000u) - 1.0f;
    }
};
__device__ static void coordinates_fl(const float n[3], float to[9]) {
    float sign = copysignf(1.0f, n[2]);
    const float a = -1.0f / (sign + n[2]);
    const float b = n[0] * n[1] * a;
    to[0] = 1.0f + sign * n[0] * n[0] * a; to[1] = sign * b; to[2] = -sign * n[0];
    to[3] = b; to[4] = sign + n[1] * n[1] * a; to[5] = -n[1];
    to[6] = n[0]; to[7] = n[1]; to[8] = n[2];
}
__global__ void __launch_bounds__(256)
hemi_gen_batched_kernel(int K, HemiGenArgs a, char* __restrict__ staging, size_t per) {
    extern __shared__ float u[];   // the stream's 10 draws per position, in draw order
    const int npos = K / 8;
    const int b = blockIdx.x;
    if (threadIdx.x == 0) {
        Pcg32Dev rng;
        rng.seed(a.seed[b], 0xda3e39cb94b95bdbULL);
        for (int i = 0; i < a.skip; ++i) (void)rng.next_uint();
        for (int i = 0; i < 10 * npos; ++i) u[i] = rng.next_float();
    }
    __syncthreads();
    const double PI = 3.14159265358979323846;
    char* blk = staging + per * (size_t)b;
    float* pw = (float*)blk;
    float* pm = (float*)(blk + 4 * (size_t)K);
    float* pc = (float*)(blk + 28 * (size_t)K);
    float* pb = (float*)(blk + 128 * (size_t)K);
    float* pd = (float*)(blk + 228 * (size_t)K);
    const float maxRadiusSqr = (float)10.644640675668422;   // chi2(6).quantile(0.9)
    const float minDist = a.dist[b];
    const float widthVarSqr = (float)(0.5 * (double)minDist * (double)minDist / (double)maxRadiusSqr);
    const float depthVarSqr = a.depth_prior * a.depth_prior / maxRadiusSqr;
    const float nThetas = 2.0f, nPhis = 4.0f;
    const float directionalInit = 1.0f / (nThetas * nPhis);
    const float dcov = (float)(2.0 * PI * (double)directionalInit);
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
        const int pi = k >> 3, ti = (k >> 2) & 1, fi = k & 3;
        const float* p = a.pos + 3 * ((size_t)npos * b + pi);
        const float* n = a.nrm + 3 * ((size_t)npos * b + pi);
        float to[9];
        coordinates_fl(n, to);
        const float* s = to;
        const float* t = to + 3;
        const float* ud = u + 10 * pi + 5 * ti;   // theta draw, then the four phi draws
        float theta = 0.0f;
        for (int j = 0; j <= ti; ++j) {
            const float rn = (float)(((double)u[10 * pi + 5 * j] - 0.5) * 2e-1);
            theta = (float)((double)theta + (0.5 * PI / (double)(nThetas + 1.0f) + (double)rn));
        }
        const float cosTheta = (float)cos((double)theta);
        const float sinTheta = (float)sqrt((double)(1.0f - cosTheta * cosTheta));
        float phi = 0.0f;
        for (int j = 0; j <= fi; ++j) {
            const float rn = (float)(((double)ud[1 + j] - 0.5) * 1e-1);
            phi = (float)((double)phi + (2.0 * PI / (double)nPhis + (double)rn));
        }
        const float sinPhi = (float)sin((double)phi), cosPhi = (float)cos((double)phi);
        const float dl0 = sinTheta * cosPhi, dl1 = sinTheta * sinPhi, dl2 = cosTheta;
        float* mean = pm + 6 * k;
        for (int i = 0; i < 3; ++i) mean[i] = p[i];
        for (int i = 0; i < 3; ++i) mean[3 + i] = (s[i] * dl0 + t[i] * dl1) + n[i] * dl2;
        float* cov = pc + 25 * k;
        float* bp = pb + 25 * k;
        for (int i = 0; i < 25; ++i) {
            cov[i] = (i % 6 == 0) ? 1.0f : 0.0f;
            bp[i] = (i % 6 == 0) ? 1.0f : 0.0f;
        }
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                cov[5 * i + j] = (s[i] * s[j] * widthVarSqr + t[i] * t[j] * widthVarSqr) + n[i] * n[j] * depthVarSqr;
                bp[5 * i + j] = s[i] * s[j] * 1e-4f + t[i] * t[j] * 1e-4f + n[i] * n[j] * 1e-4f;
            }
        cov[18] = dcov; cov[24] = dcov;
        bp[18] = 1e-5f; bp[24] = 1e-5f;
        pw[k] = (float)(1.0 / (double)K);   // 1.0f / (float)K, correctly rounded
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) pd[9 * k + 3 * i + j] = n[i] * n[j] * 1e-6f;
    }
}

hipError_t launch_hemi_gen_batched(int n, int K, const float* pos, const float* nrm, const float* dist,
                                   const uint64_t* seed, int skip, float depth_prior, void* staging, size_t per,
                                   hipStream_t st) {
    const HemiGenArgs a{pos, nrm, dist, seed, skip, depth_prior};
    const int threads = K < 64 ? 64 : (K > 256 ? 256 : K);
    hipLaunchKernelGGL(hemi_gen_batched_kernel, dim3((unsigned)n), dim3(threads), sizeof(float) * 10 * (size_t)(K / 8),
                       st, K, a, (char*)staging, per);
    return hipGetLastError();
}

hipError_t launch_set_all_batched(int n, int K, int Kp, const void* tab, const void* staging, size_t per, float norm5,
                                  hipStream_t st) {
    const int threads = Kp < 64 ? 64 : (Kp > 512 ? 512 : Kp);
    hipLaunchKernelGGL(set_all_batched_kernel, dim3((unsigned)n), dim3(threads), 0, st, K, Kp, (const InitDesc*)tab,
                       (const char*)staging, per, norm5);
    return hipGetLastError();
}

// dst[i][0 .. bytes) = src[i][0 .. bytes) for n pairs (16-byte aligned), one workgroup per pair
__global__ void __launch_bounds__(256)
copy_many_kernel(const uint4* const* __restrict__ src, uint4* const* __restrict__ dst, size_t words) {
    const uint4* s = src[blockIdx.x];
    uint4* d = dst[blockIdx.x];
    for (size_t i = threadIdx.x; i < words; i += blockDim.x) d[i] = s[i];
}

// out[i] = *src[i] (one scalar of each of n mixtures: sdmm_iterations_run)
__global__ void gather_f64_kernel(const double* const* __restrict__ src, int n, double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = *src[i];
}
hipError_t launch_gather_f64(const void* src_tab, int n, double* out, hipStream_t st) {
    hipLaunchKernelGGL(gather_f64_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       (const double* const*)src_tab, n, out);
    return hipGetLastError();
}

hipError_t launch_copy_many(int n, const void* src_tab, const void* dst_tab, size_t bytes, hipStream_t st) {
    hipLaunchKernelGGL(copy_many_kernel, dim3((unsigned)n), dim3(256), 0, st, (const uint4* const*)src_tab,
                       (uint4* const*)dst_tab, bytes / 16);
    return hipGetLastError();
}

// n mixtures carved from one slab at a fixed byte stride: mixture i's arrays
// are mixture 0's shifted by i * stride (blockIdx.y = i)
template <class T>
__device__ __forceinline__ T* shifted(T* p, size_t bytes) {
    return p ? (T*)((char*)p + bytes) : p;
}
__global__ void init_state_many_kernel(int K, InitScalars a, float eps, double* sc, float* bp, float* bd,
                                       size_t stride) {
    const size_t off = (size_t)blockIdx.y * stride;
    sc = shifted(sc, off); bp = shifted(bp, off); bd = shifted(bd, off);
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k == 0)
        for (int i = 0; i < SC_COUNT; ++i) sc[i] = a.v[i];
    if (k >= K) return;
    for (int i = 0; i < 25; ++i) bp[25 * k + i] = (i % 6 == 0) ? a.bprior[i / 6] : 0.0f;
    for (int i = 0; i < 9; ++i) bd[9 * k + i] = (i % 4 == 0) ? eps : 0.0f;
}
__global__ void __launch_bounds__(256)
pack_many_kernel(int K, int Kp, CanonDev C, float* ep, float* gp, float norm5, size_t stride) {
    const size_t off = (size_t)blockIdx.x * stride;
    C.weights = shifted(C.weights, off); C.cdf = shifted(C.cdf, off); C.mean = shifted(C.mean, off);
    C.cov = shifted(C.cov, off); C.to = shifted(C.to, off); C.cholL = shifted(C.cholL, off);
    C.cholLInv = shifted(C.cholLInv, off); C.detInv = shifted(C.detInv, off);
    C.muPremult = shifted(C.muPremult, off); C.condCov = shifted(C.condCov, off); C.margL = shifted(C.margL, off);
    C.margDetInv = shifted(C.margDetInv, off); C.condL = shifted(C.condL, off);
    C.condLInv = shifted(C.condLInv, off); C.condDetInv = shifted(C.condDetInv, off);
    C.valid = shifted(C.valid, off);
    ep = shifted(ep, off);
    gp = shifted(gp, off);
    for (int kk = threadIdx.x; kk < Kp; kk += blockDim.x) pack_component(kk, K, Kp, C, ep, gp, norm5);
}

hipError_t launch_init_pack_many(int n, int K, int Kp, const double* scal, const float* bprior, float eps,
                                 double* sc, float* bp, float* bd, const CanonDev& C, float* ep, float* gp,
                                 float norm5, size_t stride, hipStream_t st) {
    InitScalars a;
    for (int i = 0; i < SC_COUNT; ++i) a.v[i] = scal[i];
    for (int i = 0; i < 5; ++i) a.bprior[i] = bprior[i];
    hipLaunchKernelGGL(init_state_many_kernel, dim3((unsigned)((K + 63) / 64), (unsigned)n), dim3(64), 0, st, K, a,
                       eps, sc, bp, bd, stride);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pack_many_kernel, dim3((unsigned)n), dim3(256), 0, st, K, Kp, C, ep, gp, norm5, stride);
    return hipGetLastError();
}

hipError_t launch_init_state(int K, const double* scal, const float* bprior, float eps, double* sc, float* bp,
                             float* bd, hipStream_t st) {
    InitScalars a;
    for (int i = 0; i < SC_COUNT; ++i) a.v[i] = scal[i];
    for (int i = 0; i < 5; ++i) a.bprior[i] = bprior[i];
    hipLaunchKernelGGL(init_state_kernel, dim3((unsigned)((K + 63) / 64)), dim3(64), 0, st, K, a, eps, sc, bp, bd);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
hipError_t launch_set_f64(double* p, double v, hipStream_t st) {
    hipLaunchKernelGGL(set_f64_kernel, dim3(1), dim3(1), 0, st, p, v);
    return hipGetLastError();
}

hipError_t launch_set_all(int K, int Kp, const double* mean, const double* cov, const CanonDev& C,
                          float* ep, float* gp, float norm5, hipStream_t st) {
    const int threads = Kp < 64 ? 64 : (Kp > 512 ? 512 : Kp);
    hipLaunchKernelGGL(set_all_kernel, dim3(1), dim3(threads), 0, st, K, Kp, mean, cov, C, ep, gp, norm5);
    return hipGetLastError();
}

hipError_t launch_pack_all(int K, int Kp, const CanonDev& C, float* ep, float* gp, float norm5,
                           hipStream_t st) {
    hipLaunchKernelGGL(pack_all_kernel, dim3(1), dim3(256), 0, st, K, Kp, C, ep, gp, norm5);
    return hipGetLastError();
}

// scratch: 3K doubles; count: a zeroed counter (self-re-arming: atomicInc wraps).
hipError_t launch_mstep(int K, int Kp, const double* stats, int64_t nSamples, const CanonDev& C,
                        const EmStateDev& S, float* ep, float* gp, float norm5, double* newW, unsigned* count,
                        hipStream_t st) {
    if (Kp > 512 || K > Kp) return hipErrorInvalidValue;
    hipLaunchKernelGGL(mstep_spread_kernel, dim3((unsigned)((Kp + 63) / 64)), dim3(128), 0, st, K, Kp, stats,
                       nSamples, C, S, ep, gp, norm5, newW, count);
    return hipGetLastError();
}

hipError_t launch_mstep_batched(int K, int Kp, const MixDesc* mixes, int n_mix, float norm5, hipStream_t st) {
    if (n_mix <= 0) return hipSuccess;
    const int threads = Kp < 64 ? 64 : (Kp > 512 ? 512 : Kp);
    hipLaunchKernelGGL(mstep_batched_kernel, dim3(n_mix), dim3(threads), (sizeof(double) + sizeof(int) + sizeof(float)) * (size_t)K,
                       st, K, Kp, mixes, norm5);
    return hipGetLastError();
}

}  // namespace sdmm
