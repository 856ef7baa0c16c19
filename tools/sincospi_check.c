// Host check of the step kernel's sin/cos(pi t) (qcart_kernels.hpp sincospi_unit, same operations in C with
// fma/rint): 2e7 Box-Muller angles t = 2 u2 against long double, and libm on the rounded 2 pi u2 beside it.
//   gcc -O2 -o /tmp/sincospi_check tools/sincospi_check.c -lm && /tmp/sincospi_check [draws]
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
static void scp(double t, double* s, double* c) {
    const double n = rint(2.0 * t);
    const double r = fma(-0.5, n, t);
    const double x = r * 3.141592653589793, z = x * x;
    double ps = 2.8114572543455206e-15;
    ps = fma(ps, z, -7.647163731819816e-13);
    ps = fma(ps, z, 1.6059043836821613e-10);
    ps = fma(ps, z, -2.505210838544172e-08);
    ps = fma(ps, z, 2.7557319223985893e-06);
    ps = fma(ps, z, -0.0001984126984126984);
    ps = fma(ps, z, 0.008333333333333333);
    ps = fma(ps, z, -0.16666666666666666);
    const double S = fma(x * z, ps, x);
    double pc = -1.5619206968586225e-16;
    pc = fma(pc, z, 4.779477332387385e-14);
    pc = fma(pc, z, -1.1470745597729725e-11);
    pc = fma(pc, z, 2.08767569878681e-09);
    pc = fma(pc, z, -2.755731922398589e-07);
    pc = fma(pc, z, 2.48015873015873e-05);
    pc = fma(pc, z, -0.001388888888888889);
    pc = fma(pc, z, 0.041666666666666664);
    const double C = fma(z * z, pc, fma(-0.5, z, 1.0));
    const int q = (int)n & 3;
    *s = q == 0 ? S : q == 1 ? C : q == 2 ? -S : -C;
    *c = q == 0 ? C : q == 1 ? -S : q == 2 ? -C : S;
}
int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 20000000;
    uint64_t st = 88172645463325252ull; double ms = 0, mc = 0, msr = 0;
    for (long i = 0; i < n; ++i) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        const double u2 = ((double)(st >> 11) + 0.5) * 0x1.0p-53;
        double s, c; scp(2.0 * u2, &s, &c);
        const long double al = 2.0L * 3.14159265358979323846264338327950288L * (long double)u2;
        const double ds = fabs((double)((long double)s - sinl(al))), dc = fabs((double)((long double)c - cosl(al)));
        const double a = 2 * M_PI * u2;
        const double ls = fabs((double)((long double)sin(a) - sinl(al))), lc = fabs((double)((long double)cos(a) - cosl(al)));
        if (ls > msr) msr = ls; if (lc > msr) msr = lc;
        if (ds > ms) ms = ds; if (dc > mc) mc = dc;
    }
    // exact quadrant points and tiny args
    double s, c; scp(0.5, &s, &c); printf("t=.5: %g %g\n", s, c); scp(1e-300, &s, &c); printf("tiny: %g %g\n", s, c);
    printf("mine vs exact: sin %.3g cos %.3g; libm(2pi u2 rounded) vs exact %.3g\n", ms, mc, msr);
}
