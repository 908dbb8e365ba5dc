// Accuracy of the LSTM-cell transcendentals (common.h sigmoid_cell / tanh_cell) against fp64, next
// to the libm-accurate forms (sigmoidf_ / tanhf): max and mean error in fp32 ulps of the exact
// result, max absolute error, max relative error where |f| > 1e-3, over every fp32 value in
// [-30, 30] with a stride (plus all of [-1, 1] at a finer stride); tails: absolute error <= 5e-7.  Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/mathcheck.hip -o tools/mathcheck.bin
#include "../i-admm-lstm_amd/csrc/common.h"
#include <cstdio>
#include <cmath>
#include <vector>
#include <cstring>

using namespace iadmm;

__global__ void eval(int64_t n, const float* x, float* out, unsigned* packed_mismatch) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    out[4 * i + 0] = sigmoid_cell(v);
    out[4 * i + 1] = sigmoidf_(v);
    out[4 * i + 2] = tanh_cell(v);
    out[4 * i + 3] = tanhf(v);
    // the packed forms must reproduce the scalar ones bit for bit
    const float w = x[(i + 1) % n];
    const float2v sp = sigmoid_cell2(float2v{v, w}), tp = tanh_cell2(float2v{v, w});
    const bool bad = __float_as_uint(sp.x) != __float_as_uint(sigmoid_cell(v)) ||
                     __float_as_uint(sp.y) != __float_as_uint(sigmoid_cell(w)) ||
                     __float_as_uint(tp.x) != __float_as_uint(tanh_cell(v)) ||
                     __float_as_uint(tp.y) != __float_as_uint(tanh_cell(w));
    if (bad) atomicAdd(packed_mismatch, 1u);
  }
}

static double ulp_err(float got, double ref) {
  if (ref == 0.0) return got == 0.f ? 0.0 : 1e30;
  int e;
  frexp(ref, &e);                      // |ref| = f 2^e, f in [0.5,1)
  double ulp = ldexp(1.0, e - 24);     // fp32 ulp at |ref|
  if (fabs(ref) < ldexp(1.0, -126)) ulp = ldexp(1.0, -149);
  return fabs((double)got - ref) / ulp;
}

int main() {
  std::vector<float> xs;
  uint32_t lo, hi;
  for (float a = -30.f; a <= 30.f;) { xs.push_back(a); float b = nextafterf(a, 40.f); for (int k = 0; k < 97; ++k) b = nextafterf(b, 40.f); a = b; }
  for (float a = -1.f; a <= 1.f;) { xs.push_back(a); float b = nextafterf(a, 2.f); for (int k = 0; k < 7; ++k) b = nextafterf(b, 2.f); a = b; }
  // the tails and the specials: exact results there are 0 / 1 / -1 (or denormal), any NaN is a bug
  for (float a = 30.f; a <= 1e30f; a *= 1.37f) { xs.push_back(a); xs.push_back(-a); }
  xs.push_back(INFINITY); xs.push_back(-INFINITY); xs.push_back(3.4e38f); xs.push_back(-3.4e38f);
  (void)lo; (void)hi;
  const int64_t n = xs.size();
  float *dx, *dout;
  unsigned* dbad;
  hipMalloc(&dx, n * 4); hipMalloc(&dout, n * 16); hipMalloc(&dbad, 4);
  hipMemset(dbad, 0, 4);
  hipMemcpy(dx, xs.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(eval, dim3(4096), dim3(256), 0, 0, n, dx, dout, dbad);
  unsigned bad = 0;
  hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
  printf("packed vs scalar forms: %u mismatching points\n", bad);
  std::vector<float> out(4 * n);
  hipMemcpy(out.data(), dout, n * 16, hipMemcpyDeviceToHost);
  {  // no NaN from a non-NaN input, and the limits are reached
    int bad = 0;
    for (int64_t i = 0; i < n; ++i)
      for (int f = 0; f < 4; ++f)
        if (std::isnan(out[4 * i + f])) ++bad;
    printf("NaN outputs from non-NaN inputs: %d\n", bad);
  }
  const char* names[4] = {"sigmoid_cell", "sigmoidf_ (1/(1+expf))", "tanh_cell", "tanhf (ocml)"};
  for (int f = 0; f < 4; ++f) {
    double mx = 0, sum = 0, amx = 0, rmx = 0; float worst = 0;
    for (int64_t i = 0; i < n; ++i) {
      const double v = xs[i];
      if (!(fabs(v) <= 30.0)) {  // tails: absolute error only
        const double ref = f < 2 ? 1.0 / (1.0 + exp(-v)) : tanh(v);
        if (fabs((double)out[4 * i + f] - ref) > 5e-7) { printf("tail error %s x=%g got %g\n", names[f], v, out[4*i+f]); }
        continue;
      }
      const double ref = f < 2 ? 1.0 / (1.0 + exp(-v)) : tanh(v);
      const double e = ulp_err(out[4 * i + f], ref);
      amx = fmax(amx, fabs((double)out[4 * i + f] - ref));
      if (fabs(ref) > 1e-3) rmx = fmax(rmx, fabs((double)out[4 * i + f] - ref) / fabs(ref));
      sum += e;
      if (e > mx) { mx = e; worst = xs[i]; }
    }
    printf("%-24s max %.3f ulp (at x=%.9g)  mean %.4f ulp  max abs %.3g  max rel (|f|>1e-3) %.3g  over %lld points\n",
           names[f], mx, worst, sum / n, amx, rmx, (long long)n);
  }
  return 0;
}
