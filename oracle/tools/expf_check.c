/* TEST INFRASTRUCTURE: exhaustive check of orc_expf against this machine's libm expf
 * over every float in [lo, hi) (default: [0, 8), which covers 0.25*r2 for r2 <= 40/3). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../letkf_oracle.h"
int main(int argc, char **argv)
{
  float lo = argc > 1 ? strtof(argv[1], 0) : 0.0f, hi = argc > 2 ? strtof(argv[2], 0) : 8.0f;
  uint32_t a, b; memcpy(&a, &lo, 4); memcpy(&b, &hi, 4);
  long long bad = 0, n = 0;
  volatile float (*libexpf)(float) = (volatile float (*)(float))expf;
#pragma omp parallel for reduction(+ : bad, n) schedule(static, 65536)
  for (long long u = a; u < (long long)b; ++u) {
    float x; uint32_t uu = (uint32_t)u; memcpy(&x, &uu, 4);
    float r1 = orc_expf(x), r2 = libexpf(x);
    n++;
    if (memcmp(&r1, &r2, 4) != 0) { bad++; }
  }
  printf("expf_check [%g,%g): %lld values, %lld mismatches\n", lo, hi, n, bad);
  return bad != 0;
}
