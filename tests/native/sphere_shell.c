/* Exhaustive check of the RNG pre-pass's integer accept test (rfx_kernels.hip triple) against the reference's float
 * test over every triple of 15-bit draws: 2^45 (k1, k2, k3).
 *
 * Reference (src/common/Vector3.cpp:182-185): x = float(k) / (float(0x7FFF) / 2) - 1 for each of the three draws, and
 * the triple is rejected when x*x + y*y + z*z > 1 (float, left to right, no contraction).  The device decides with
 * N = (2k1 - 32767)^2 + (2k2 - 32767)^2 + (2k3 - 32767)^2 against 32767^2 and runs the float test only inside a shell
 * |N - 32767^2| <= shell.  The integer test is right outside the shell iff every float-accepted triple has
 * N < 32767^2 + shell and every float-rejected one has N > 32767^2 - shell.  This program prints the largest N of an
 * accepted triple and the smallest N of a rejected one, and the total accepted count.
 *
 * Method: for a fixed (k1, k2) and one side of k3 (k3 >= 16384: x3 > 0, or k3 <= 16383: x3 < 0), |x3| and so
 * float(x3 * x3) are nondecreasing in |2k3 - 32767| (checked below), and float addition is monotone, so the accepted
 * k3 of that side are the ones nearest the centre up to one boundary, found by bisection; the accepted triple of
 * largest N and the rejected one of smallest N sit on either side of it.
 *
 *   gcc -O2 -ffp-contract=off -fopenmp sphere_shell.c -o sphere_shell && ./sphere_shell [k1_stride]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static float X[32768], SQ[32768];
static int idx_side[2][16384]; /* k3 of each side in increasing |2k3 - 32767| */

int main(int argc, char **argv)
{
  const int stride = argc > 1 ? atoi(argv[1]) : 1;
  const float half = (float)0x7FFF / 2.0f;
  for (int k = 0; k < 32768; ++k)
  {
    volatile float q = (float)k / half; /* one rounding, then the subtraction's */
    X[k] = q - 1.0f;
    volatile float s = X[k] * X[k];
    SQ[k] = s;
  }
  for (int t = 0; t < 16384; ++t)
  {
    idx_side[0][t] = 16384 + t; /* v3 = 2t + 1 */
    idx_side[1][t] = 16383 - t; /* v3 = -(2t + 1) */
  }
  for (int sd = 0; sd < 2; ++sd)
    for (int t = 1; t < 16384; ++t)
      if (SQ[idx_side[sd][t]] < SQ[idx_side[sd][t - 1]])
      {
        printf("{\"error\": \"x^2 not monotone on side %d at %d\"}\n", sd, t);
        return 1;
      }
  const int64_t R2 = 32767LL * 32767LL;
  int64_t acc_max = -1, rej_min = INT64_MAX;
  uint64_t accepted = 0, pairs = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(max : acc_max) reduction(min : rej_min) \
    reduction(+ : accepted, pairs)
  for (int k1 = 0; k1 < 32768; k1 += stride)
  {
    const int64_t v1 = 2 * k1 - 32767;
    for (int k2 = 0; k2 < 32768; ++k2)
    {
      const int64_t v2 = 2 * k2 - 32767;
      volatile float av = SQ[k1] + SQ[k2];
      const float a = av;
      ++pairs;
      for (int sd = 0; sd < 2; ++sd)
      {
        const int *ix = idx_side[sd];
        /* T = number of accepted k3 on this side: acc(t) for t < T */
        int lo = 0, hi = 16384;
        while (lo < hi)
        {
          const int mid = (lo + hi) >> 1;
          volatile float sum = a + SQ[ix[mid]];
          if (!(sum > 1.0f))
            lo = mid + 1;
          else
            hi = mid;
        }
        accepted += (uint64_t)lo;
        const int64_t base = v1 * v1 + v2 * v2;
        if (lo > 0)
        {
          const int64_t v3 = 2 * (int64_t)ix[lo - 1] - 32767, n = base + v3 * v3;
          if (n > acc_max) acc_max = n;
        }
        if (lo < 16384)
        {
          const int64_t v3 = 2 * (int64_t)ix[lo] - 32767, n = base + v3 * v3;
          if (n < rej_min) rej_min = n;
        }
      }
    }
  }
  printf("{\"stride\": %d, \"pairs\": %llu, \"accepted\": %llu, \"r2\": %lld, \"accepted_max_n\": %lld, "
         "\"rejected_min_n\": %lld, \"shell_needed\": %lld}\n",
         stride, (unsigned long long)pairs, (unsigned long long)accepted, (long long)R2, (long long)acc_max,
         (long long)rej_min, (long long)((acc_max - R2) > (R2 - rej_min) ? (acc_max - R2) : (R2 - rej_min)));
  return 0;
}
