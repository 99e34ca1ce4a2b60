// rpoly_ref.cpp -- test harness (oracle side only): a C entry point for the reference's own
// Jenkins-Traub root finder, usac/estimator/essential/rpoly.cpp:7-230 (rpoly_ak1), which
// oracle/Makefile compiles where it lies (never copied) and links beside this file into
// oracle/_ref/librpoly_ref.so.  Five_points.cpp:143-160 calls it with the degree-10
// coefficients highest power first and keeps the roots whose imaginary part is exactly zero,
// in the order rpoly_ak1 found them; tests/test_oracle_essential.py compares that with the
// oracle's real_roots (usac_oracle.c) on the oracle's own polynomials.
#define MAXDEGREE 100
#define MDP1 MAXDEGREE + 1

void rpoly_ak1(double op[MDP1], int *Degree, double zeror[MAXDEGREE], double zeroi[MAXDEGREE]);

// a: n + 1 coefficients, ascending powers (the oracle's layout).  Writes rpoly_ak1's raw zeros
// (zr, zi: `degree` of them, in its order) and returns the degree it reports back (n, less the
// zeros it failed to find after 20 shifts, 0 for a zero leading coefficient, -1 if n > 100).
extern "C" int rpoly_ref_zeros(const double *a, int n, double *zr, double *zi) {
    double op[MDP1], r[MAXDEGREE], i[MAXDEGREE];
    if (n < 1 || n > MAXDEGREE) return -1;
    for (int k = 0; k <= n; k++) op[k] = a[n - k];  // five_points.cpp:146-148: highest power first
    int degree = n;
    rpoly_ak1(op, &degree, r, i);
    for (int k = 0; k < degree; k++) {
        zr[k] = r[k];
        zi[k] = i[k];
    }
    return degree;
}

// the reference's selection (five_points.cpp:152-156): the real zeros (zeroi == 0) in found order
extern "C" int rpoly_ref_real_roots(const double *a, int n, double *roots) {
    double zr[MAXDEGREE], zi[MAXDEGREE];
    const int degree = rpoly_ref_zeros(a, n, zr, zi);
    int k = 0;
    for (int j = 0; j < degree; j++)
        if (zi[j] == 0) roots[k++] = zr[j];
    return k;
}
