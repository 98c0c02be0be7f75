/* The C library's pow / exp / asin / acos / tan over arrays, for the host-side case builder
 * (mpas_dycore/init_atm.py).  The reference's initialisation calls these functions of the C
 * library element by element; init_atm reproduces its arithmetic with the same library, and this
 * loop does in C what np.frompyfunc(math.pow, ...) does one Python call at a time.  Built without
 * -ffast-math, so every element is one scalar call of the library function (no vector variants). */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>

void hl_pow_s(const double* x, double y, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = pow(x[i], y);
}
void hl_pow_v(const double* x, const double* y, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = pow(x[i], y[i]);
}
void hl_exp(const double* x, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = exp(x[i]);
}
void hl_asin(const double* x, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = asin(x[i]);
}
void hl_acos(const double* x, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = acos(x[i]);
}
void hl_tan(const double* x, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = tan(x[i]);
}
/* sincos: the compiled reference evaluates cos(x) and sin(x) of one argument in one basic block as a
 * single sincos() call (amdflang -O2 merges them), which differs from separate cos / sin in the last
 * bit for ~0.06 % of arguments; the restatement calls the same function where the reference's
 * compiler fuses the pair. */
void hl_sincos(const double* x, double* s, double* c, int64_t n) {
  for (int64_t i = 0; i < n; ++i) sincos(x[i], &s[i], &c[i]);
}
