// ADMM scalar schedule and the fused x/z/y update.
//
// Reference: models/lstm.py:60-63 (rho, rho_vec, alpha), :80 (+ b_h), :82-94 (xv step, x
// relaxation, z projection, dual update); models/lu.py:38-45 (Stage II variant with z
// relaxation).  Compiled with -ffp-contract=off so every a*b+c below rounds twice, exactly as
// the reference's separate tensor ops do.
#include "common.h"

namespace iadmm {

__global__ void schedule_kernel(const float* rho_param, const float* alpha_param, int64_t t,
                                float* scal) {
  if (threadIdx.x != 0) return;
  const float rho = sigmoidf_(rho_param[t]);
  const float rho_eq = rho * 1e3f;
  const float alpha = 2.0f * sigmoidf_(alpha_param[t]);
  scal[IADMM_S_RHO_IN] = rho;
  scal[IADMM_S_RHO_EQ] = rho_eq;
  scal[IADMM_S_IRHO_IN] = 1.0f / rho;
  scal[IADMM_S_IRHO_EQ] = 1.0f / rho_eq;
  scal[IADMM_S_ALPHA] = alpha;
  scal[IADMM_S_1MALPHA] = 1.0f - alpha;
  scal[6] = 0.f;
  scal[7] = 0.f;
}

__global__ void schedule_fixed_kernel(const float* in, float alpha, float* out) {
  if (threadIdx.x != 0) return;
  for (int i = 0; i < IADMM_NSCAL; ++i) out[i] = in[i];
  out[IADMM_S_ALPHA] = alpha;
  out[IADMM_S_1MALPHA] = 1.0f - alpha;
}

struct UpdArgs {
  int64_t B;
  int n, m, num_ineq, ntiles, relax_z;
  const float *part, *bh, *xv, *x, *y, *z, *zl, *zu, *scal, *rho_rows;
  float *xvo, *xo, *yo, *zo, *rhovec;
};

__global__ __launch_bounds__(256) void admm_update_kernel(UpdArgs a) {
  const int N = a.n + a.m;
  const int64_t M = a.B * (int64_t)N;
  const float rho_in = a.scal[IADMM_S_RHO_IN], rho_eq = a.scal[IADMM_S_RHO_EQ];
  const float irho_in = a.scal[IADMM_S_IRHO_IN], irho_eq = a.scal[IADMM_S_IRHO_EQ];
  const float alpha = a.scal[IADMM_S_ALPHA], oma = a.scal[IADMM_S_1MALPHA];
  const float bh = a.part ? a.bh[0] : 0.f;
  for (int64_t R = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; R < M;
       R += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = R / N;
    const int i = (int)(R - b * N);
    float xvn;
    if (a.part) {
      float s = 0.f;
      for (int tl = 0; tl < a.ntiles; ++tl) s += a.part[(int64_t)tl * M + R];  // fixed order
      xvn = a.xv[R] - (s + bh);
    } else {
      xvn = a.xv[R];  // Stage II: xv already solved
    }
    a.xvo[R] = xvn;
    if (i < a.n) {
      const int64_t k = b * a.n + i;
      a.xo[k] = alpha * xvn + oma * a.x[k];
    } else {
      const int j = i - a.n;
      const int64_t k = b * a.m + j;
      const bool ineq = j < a.num_ineq;
      float rho = ineq ? rho_in : rho_eq, irho = ineq ? irho_in : irho_eq;
      if (a.rho_rows) { rho = a.rho_rows[k]; irho = 1.0f / rho; }  // explicit rho_vec (models/lu.py)
      const float y = a.y[k], z = a.z[k];
      const float zt = z + irho * (xvn - y);
      const float zr = a.relax_z ? alpha * zt + oma * z : zt;
      const float zn = tmax(tmin(zr + irho * y, a.zu[k]), a.zl[k]);
      a.zo[k] = zn;
      a.yo[k] = y + rho * (zr - zn);
      if (a.rhovec) a.rhovec[k] = rho;
    }
  }
}

}  // namespace iadmm

using namespace iadmm;

extern "C" int iadmm_version(void) { return 11; }

extern "C" int iadmm_schedule(const float* rho_param, const float* alpha_param, int64_t t,
                              float* scal, void* stream) {
  if (!rho_param || !alpha_param || !scal || t < 0) return IADMM_E_ARG;
  hipLaunchKernelGGL(schedule_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, rho_param,
                     alpha_param, t, scal);
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_schedule_fixed_alpha(const float* scal_in, float alpha, float* scal_out,
                                          void* stream) {
  if (!scal_in || !scal_out) return IADMM_E_ARG;
  hipLaunchKernelGGL(schedule_fixed_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, scal_in,
                     alpha, scal_out);
  IADMM_CHECK_LAUNCH();
  return 0;
}

extern "C" int iadmm_admm_update(int64_t B, int64_t n, int64_t m, int64_t num_ineq,
                                 int64_t ntiles, const float* part, const float* b_h,
                                 const float* xv, const float* x, const float* y, const float* z,
                                 const float* zl, const float* zu, const float* scal,
                                 const float* rho_rows, int relax_z,
                                 float* xv_out, float* x_out, float* y_out, float* z_out,
                                 float* rho_vec, void* stream) {
  if (B <= 0 || n <= 0 || m < 0 || num_ineq < 0 || num_ineq > m) return IADMM_E_ARG;
  if (!xv || !x || !scal || !xv_out || !x_out) return IADMM_E_ARG;
  if (m > 0 && (!y || !z || !zl || !zu || !y_out || !z_out)) return IADMM_E_ARG;
  if (part && (!b_h || ntiles <= 0)) return IADMM_E_ARG;
  if (xv_out == xv || x_out == x || (m > 0 && (y_out == y || z_out == z))) return IADMM_E_ARG;
  UpdArgs a{B, (int)n, (int)m, (int)num_ineq, (int)ntiles, relax_z, part, b_h, xv, x, y, z, zl,
            zu, scal, rho_rows, xv_out, x_out, y_out, z_out, rho_vec};
  const int64_t M = B * (n + m);
  const int64_t blocks = (M + 255) / 256;
  hipLaunchKernelGGL(admm_update_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256),
                     0, (hipStream_t)stream, a);
  IADMM_CHECK_LAUNCH();
  return 0;
}
