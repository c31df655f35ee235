// Quad-split point arithmetic: one point operation spread over the 4 lanes of a quad, for serial
// point chains that a lone wave would otherwise run at one field product per step (k_msm_final's
// Horner chain, the exact batch path's z_i D_i).
#pragma once
#include <hip/hip_runtime.h>
#include "nw_point.h"

namespace nw {

NW_HD ge_p3 ge_add_p3(const ge_p3& a, const ge_p3& b) { return ge_add(a, ge_to_cached(b)); }

// The serial tail of a batch (k_msm_final's Horner over the window sums: 254 doublings + 31
// additions) is one dependent chain that every lane of the wave runs redundantly.  Splitting each
// point operation over the 4 lanes of a quad turns its independent field products into ONE SIMD
// product per lane (lane q takes operand pair q): a doubling is 1 squaring + 1 multiplication per
// lane instead of 4 + 3, an addition 3 multiplications instead of 9.  Operands are exchanged with
// DPP quad broadcasts (full-rate VALU moves); every quad ends with the full point in all 4 lanes.
template <int Q>
__device__ __forceinline__ fe fe_quad_bcast(const fe& x) {
    fe r;
#pragma unroll
    for (int k = 0; k < 10; ++k)
        r.v[k] = (uint32_t)__builtin_amdgcn_mov_dpp((int)x.v[k], Q * 0x55, 0xF, 0xF, false);
    return r;
}

// operand q (0..3) of this lane's quad position
__device__ __forceinline__ fe fe_quad_pick(const fe& a0, const fe& a1, const fe& a2, const fe& a3, uint32_t m1,
                                           uint32_t m2) {
    return fe_select_mask(fe_select_mask(a0, a1, m1), fe_select_mask(a2, a3, m1), m2);
}

__device__ __forceinline__ ge_p3 ge_quad_gather(const fe& prod) {
    ge_p3 r;
    r.X = fe_quad_bcast<0>(prod);
    r.Y = fe_quad_bcast<1>(prod);
    r.Z = fe_quad_bcast<2>(prod);
    r.T = fe_quad_bcast<3>(prod);
    return r;
}

// 2p (dbl-2008-hwcd, as ge_dbl): squarings X^2, Y^2, Z^2, (X+Y)^2 on lanes 0..3, then the products
// X = xr tr, Y = yr zr, Z = zr tr, T = xr yr.
__device__ __forceinline__ ge_p3 ge_dbl_quad(const ge_p3& p) {
    const uint32_t q = threadIdx.x & 3u;
    const uint32_t m1 = lane_mask(q & 1u), m2 = lane_mask(q & 2u);
    const fe sq = fe_sq(fe_quad_pick(p.X, p.Y, p.Z, fe_add(p.X, p.Y), m1, m2));
    const fe xx = fe_quad_bcast<0>(sq), yy = fe_quad_bcast<1>(sq), zz = fe_quad_bcast<2>(sq);
    const fe s = fe_quad_bcast<3>(sq);
    const fe yr = fe_add(yy, xx);        // k=2
    const fe zr = fe_sub(yy, xx);        // tight
    const fe xr = fe_sub(s, yr);         // tight
    const fe tr = fe_sub(fe_add(zz, zz), zr);
    return ge_quad_gather(fe_mul(fe_quad_pick(xr, yr, zr, xr, m1, m2), fe_quad_pick(tr, zr, tr, yr, m1, m2)));
}

// a + b (both extended; the formulas of ge_add(a, ge_to_cached(b))): (Ya-Xa)(Yb-Xb),
// (Ya+Xa)(Yb+Xb), Ta Tb, Za Zb on lanes 0..3; 2d Ta Tb on every lane; then the four products.
// Here b is given as this lane's operand only (lane q: operand q of b, ge_quad_operand), so a
// table of b's keeps 10 words per lane instead of the whole point.
__device__ __forceinline__ ge_p3 ge_add_quad_v(const ge_p3& a, const fe& v) {
    const uint32_t q = threadIdx.x & 3u;
    const uint32_t m1 = lane_mask(q & 1u), m2 = lane_mask(q & 2u);
    const fe u = fe_quad_pick(fe_sub(a.Y, a.X), fe_add(a.Y, a.X), a.T, a.Z, m1, m2);
    const fe pr = fe_mul(u, v);
    const fe a1 = fe_quad_bcast<0>(pr), b1 = fe_quad_bcast<1>(pr), tt = fe_quad_bcast<2>(pr);
    const fe zz = fe_quad_bcast<3>(pr);
    const fe c1 = fe_mul(tt, fe_from_const(FE_D2));
    const fe d = fe_add(zz, zz);
    const fe e = fe_sub(b1, a1);
    const fe h = fe_add(b1, a1);
    const fe f = fe_sub(d, c1);
    const fe g = fe_add(d, c1);
    return ge_quad_gather(fe_mul(fe_quad_pick(e, g, g, e, m1, m2), fe_quad_pick(f, h, f, h, m1, m2)));
}

// Lane q's operand of b in ge_add_quad_v: Yb - Xb, Yb + Xb (carried), Tb, Zb.
__device__ __forceinline__ fe ge_quad_operand(const ge_p3& b) {
    const uint32_t q = threadIdx.x & 3u;
    const uint32_t m1 = lane_mask(q & 1u), m2 = lane_mask(q & 2u);
    return fe_quad_pick(fe_sub(b.Y, b.X), fe_carry(fe_add(b.Y, b.X)), b.T, b.Z, m1, m2);
}

__device__ __forceinline__ ge_p3 ge_add_quad(const ge_p3& a, const ge_p3& b) {
    return ge_add_quad_v(a, ge_quad_operand(b));
}

}  // namespace nw
