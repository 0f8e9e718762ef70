// mbls_xyzz.hpp -- XYZZ coordinates for the bucket accumulation (x = X/ZZ, y = Y/ZZZ, with
// ZZ^3 = ZZZ^2 for every point the formulas below produce).
//
// Mixed addition madd-2008-s costs 6M + 2S + one lazy product-sum; the Jacobian madd-2007-bl
// of mbls_curve.hpp costs 6M + 4S + one (its S2 = Y2 Z1 Z1^2 is two products, Z3 one square):
// about 15% fewer mads per contribution in k_accumulate (G1: 2604 vs 3048).  A chunk partial
// is converted to Jacobian when it is stored (2M + 2S), so everything downstream is unchanged.
// Formulas: hyperelliptic.org EFD, short Weierstrass a = 0, xyzz (madd-2008-s, mdbl-2008-s-1).
// The reference accumulates in Jacobian (point.cuh:803-912).
#pragma once
#include "mbls_curve.hpp"

namespace mbls {

template <class F>
struct XYZZ {
    F x, y, zz, zzz;
    MBLS_DEV bool is_inf() const { return zz.is_zero(); }
    MBLS_DEV static XYZZ inf() { return {F::one(), F::one(), F::zero(), F::zero()}; }
};

// 2Q for affine Q (mdbl-2008-s-1 with ZZ1 = ZZZ1 = 1)
template <class F>
MBLS_DEV XYZZ<F> xyzz_mdbl(const Affine<F>& q) {
    F U = dbl(q.y);
    F V = sqr(U);
    F W = U * V;
    F S = q.x * V;
    F X2 = sqr(q.x);
    F M = dbl(X2) + X2;
    XYZZ<F> r;
    r.x = sqr(M) - dbl(S);
    r.y = mul_sum(M, S - r.x, neg(W), q.y);
    r.zz = V;
    r.zzz = W;
    return r;
}

// P + Q for affine Q (madd-2008-s); P == Q doubles Q, P == -Q gives the identity
template <class F>
MBLS_DEV XYZZ<F> xyzz_madd(const XYZZ<F>& p, const Affine<F>& q) {
    if (q.is_inf()) return p;
    if (p.is_inf()) return {q.x, q.y, F::one(), F::one()};
    F U2 = q.x * p.zz;
    F S2 = q.y * p.zzz;
    F P = U2 - p.x;
    F R = S2 - p.y;
    if (P.is_zero()) {
        if (R.is_zero()) return xyzz_mdbl(q);
        return XYZZ<F>::inf();
    }
    F PP = sqr(P);
    F PPP = P * PP;
    F Q = p.x * PP;
    XYZZ<F> r;
    r.x = sqr(R) - PPP - dbl(Q);
    r.y = mul_sum(R, Q - r.x, neg(p.y), PPP);
    r.zz = p.zz * PP;
    r.zzz = p.zzz * PPP;
    return r;
}

// Jacobian with lambda = ZZZ (= Z^3): X' = X ZZ^2, Y' = Y ZZZ^2, Z' = ZZZ, because
// X'/Z'^2 = X ZZ^2 / ZZ^3 and Y'/Z'^3 = Y / ZZZ.  The identity (ZZ = ZZZ = 0) maps to Z' = 0.
template <class F>
MBLS_DEV Jacobian<F> xyzz_to_jac(const XYZZ<F>& p) {
    if (p.is_inf()) return Jacobian<F>::inf();
    Jacobian<F> r;
    r.x = p.x * sqr(p.zz);
    r.y = p.y * sqr(p.zzz);
    r.z = p.zzz;
    return r;
}

}  // namespace mbls
