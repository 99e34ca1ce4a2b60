// mblock_ref.cpp -- test harness (oracle side only): evaluates the reference's own generated
// polynomial matrix of the 5-point solver (usac/estimator/essential/mblock.hpp, compiled from
// /root/reference where it lies, never copied).  mblock.hpp is a bare block of 200
// `M(r,c)[k] = ...;` assignments over the null-basis entries e00..e38 (five_points.cpp:69-104
// names them: eJK = entry K of vt row 5 + J) that five_points.cpp:111 includes inside
// Solve5PointEssential; here it is included inside a function of our own that supplies the
// names and a minimal PolyMatrix (the reference's polynomial.hpp pulls in OpenCV through
// precomp.hpp).  Pins the oracle's e5_matrix (usac_oracle.c) -- built into oracle/_ref/ by
// oracle/Makefile when the reference is present; tests/test_oracle_essential.py compares.
#include <cstddef>
#include <vector>

namespace {

// coefficients of z^k, grown on write (the reference's Polynomial::operator[] zero-extends)
struct Poly {
    std::vector<double> c;
    double &operator[](int k) {
        if ((int)c.size() <= k) c.resize(k + 1, 0.0);
        return c[k];
    }
    // Polynomial::Eval (polynomial.hpp): ascending powers, the power updated by a multiply
    double eval(double z) const {
        double ret = 0.0, t = 1.0;
        for (std::size_t i = 0; i < c.size(); i++) {
            ret += c[i] * t;
            t *= z;
        }
        return ret;
    }
};

struct PolyMatrix {
    Poly p[10][10];
    Poly &operator()(int r, int col) { return p[r][col]; }
};

void fill(const double *N, PolyMatrix &M) {
    const double e00 = N[0], e01 = N[1], e02 = N[2], e03 = N[3], e04 = N[4], e05 = N[5], e06 = N[6], e07 = N[7],
                 e08 = N[8];
    const double e10 = N[9], e11 = N[10], e12 = N[11], e13 = N[12], e14 = N[13], e15 = N[14], e16 = N[15],
                 e17 = N[16], e18 = N[17];
    const double e20 = N[18], e21 = N[19], e22 = N[20], e23 = N[21], e24 = N[22], e25 = N[23], e26 = N[24],
                 e27 = N[25], e28 = N[26];
    const double e30 = N[27], e31 = N[28], e32 = N[29], e33 = N[30], e34 = N[31], e35 = N[32], e36 = N[33],
                 e37 = N[34], e38 = N[35];
#include "mblock.hpp"
}

}  // namespace

// M(z) of the null basis N (4 x 9 row-major: N0..N3 = vt rows 5..8), 10 x 10 row-major: row r =
// constraint, column = monomial [x^3, y^3, x^2 y, x y^2, x^2, y^2, x y, x, y, 1]
extern "C" void mblock_ref_eval(const double *N, double z, double *out) {
    PolyMatrix M;
    fill(N, M);
    for (int r = 0; r < 10; r++)
        for (int col = 0; col < 10; col++) out[10 * r + col] = M(r, col).eval(z);
}

// the polynomial coefficients themselves: out[(10 r + col) * 4 + k] = coefficient of z^k (k <= 3)
extern "C" void mblock_ref_coeffs(const double *N, double *out) {
    PolyMatrix M;
    fill(N, M);
    for (int r = 0; r < 10; r++)
        for (int col = 0; col < 10; col++)
            for (int k = 0; k < 4; k++)
                out[(10 * r + col) * 4 + k] = k < (int)M(r, col).c.size() ? M(r, col).c[k] : 0.0;
}
