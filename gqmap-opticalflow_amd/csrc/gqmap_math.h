// gqmap_math.h -- per-element arithmetic of one QGMAP iteration.
//
// This header is the arithmetic specification of the hot path: the HIP
// kernel (gqmap_engine.hip) and the CPU emulator (oracle/gqmap_emul.cpp,
// test infrastructure) both include it, so a node/edge gradient evaluates to
// the same bits on both sides.  Rules that make that hold:
//   * every fused multiply-add is an explicit fma(); both sides compile with
//     -ffp-contract=off, so nothing else is contracted;
//   * sqrt and division are IEEE correctly rounded on both sides
//     (GQ_SQRT is provided by the includer: the device form is LLVM's
//     correctly rounded f64 sequence without its denormal rescaling);
//   * log/exp are the deterministic routines below (no libm);
//   * sums over pixels are exact (128-bit fixed point), so their value does
//     not depend on the order in which tiles, waves or threads add them.
//
// The includer defines GQ_HD (e.g. `__device__ __forceinline__` or `inline`),
// GQ_SQRT(x) for double and float, GQ_UNROLL2, GQ_NODE_UNROLL, GQ_UNROLL_FULL and
// GQ_PAIR_UNROLL_K(n) (loop-unroll pragmas or nothing), makes fma/fmin/fmax/floorf/fminf/fmaxf visible for float and double, then includes
// this file.
//
// Reference lines this arithmetic restates: node_pot / edge_pot
// (gqmap_gpu_mixture.m:156-182), node/edge_grad_spectral (:87-146), super
// node sum (gqmap_gpuSuper_mix_entropy.m:94-105), coarse-to-fine level
// (legacy/gqmap_ctf.m:79-150).
#pragma once
#include <stdint.h>
#include <string.h>

#include <type_traits>

namespace gq {

#ifndef GQ_M_PI
#define GQ_M_PI 3.14159265358979323846
#define GQ_M_SQRT2 1.41421356237309504880
#endif

constexpr int TAB_STRIDE = 256;  // quadrature points the table holds (K2 <= 256)
constexpr int NTAB = 8;          // entries per quadrature point, rows below
// Table rows: the node XI, XJ, the weight W = WIWJ and W times the basis
// monomials.  Rows a packed fp32 update reads as one pair are adjacent
// ((W, W a), (W XI, W XJ), (W m, W x)).
constexpr int T_XI = 0, T_XJ = 1, T_W = 2, T_WA = 3, T_WXI = 4, T_WXJ = 5, T_WM = 6, T_WX = 7;
//   WA = W (XI^2 + XJ^2), WM = W (XI^2 - XJ^2), WX = W XI XJ
// Table entry r of quadrature point k.  Point-major: the 8 entries of a
// point are contiguous, so a wave-uniform point costs one scalar load
// (s_load_dwordx8 / x16) instead of eight.
#ifdef __HIPCC__
__host__ __device__
#endif
constexpr int tab_at(int r, int k) { return k * NTAB + r; }

// ---------------------------------------------------------------------------
// deterministic log / exp (classic fdlibm-style reductions, < 1 ulp)
// ---------------------------------------------------------------------------
GQ_HD uint64_t bits_of(double x)
{
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}
GQ_HD double from_bits(uint64_t u)
{
    double x;
    memcpy(&x, &u, 8);
    return x;
}

// natural log for positive normal x (callers pass sqrt(1-p^2)*o1*o2 > 0)
GQ_HD double gq_log(double x)
{
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    uint64_t u = bits_of(x);
    int k = (int)((u >> 52) & 0x7ff) - 1023;
    u = (u & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL;  // m in [1,2)
    double m = from_bits(u);
    if (m > 1.4142135623730951) {
        m = m * 0.5;
        k += 1;
    }
    const double f = m - 1.0;
    const double s = f / (2.0 + f);
    const double z = s * s, w = z * z;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    const double dk = (double)k;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

// exp for |x| <= 700 (softmax of w in [-300,300]; normal pdf tails flush to 0)
GQ_HD double gq_exp(double x)
{
    if (x < -745.0) return 0.0;
    if (x > 709.0) x = 709.0;
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 inv_ln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    const double kd = x * inv_ln2 + (x < 0 ? -0.5 : 0.5);
    const int k = (int)kd;  // round half away from zero
    const double hi = x - (double)k * ln2_hi, lo = (double)k * ln2_lo;
    const double r = hi - lo;
    const double t = r * r;
    const double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    const double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    // y * 2^k, split so subnormal results are exact scalings
    int k1 = k / 2, k2 = k - k1;
    return y * from_bits((uint64_t)(1023 + k1) << 52) * from_bits((uint64_t)(1023 + k2) << 52);
}

GQ_HD double gq_logf_via_double(float x) { return gq_log((double)x); }

template <typename R>
GQ_HD R gq_logr(R x);
template <>
GQ_HD double gq_logr<double>(double x) { return gq_log(x); }
template <>
GQ_HD float gq_logr<float>(float x) { return (float)gq_log((double)x); }

// ---------------------------------------------------------------------------
// exact, order-independent sums: value * 2^64 as a 128-bit integer
// ---------------------------------------------------------------------------
typedef __int128 fix128;

GQ_HD fix128 to_fix(double x)
{
    // x = mant * 2^(exp-1075) with a 53-bit integer mantissa (normal doubles)
    const uint64_t u = bits_of(x);
    const int bexp = (int)((u >> 52) & 0x7ff);
    if (bexp == 0x7ff) return (fix128)0;  // inf/nan: excluded (flagged separately)
    int64_t mant = (int64_t)(u & 0x000fffffffffffffULL);
    int e = bexp - 1075;
    if (bexp) mant |= (int64_t)1 << 52;
    else e = -1074;
    const int shift = e + 64;  // scale by 2^64
    fix128 v;
    if (shift >= 0) {
        const int s = shift > 72 ? 72 : shift;  // saturate |x| >= 2^61
        v = (fix128)mant << s;
    } else if (shift > -64) {
        v = (fix128)(mant >> (-shift));  // truncation toward zero of |x|
    } else {
        v = 0;
    }
    return (u >> 63) ? -v : v;
}

GQ_HD double from_fix(fix128 v)
{
    const int64_t hi = (int64_t)(v >> 64);
    const uint64_t lo = (uint64_t)v;
    return (double)hi + (double)lo * 5.42101086242752217004e-20;  // lo * 2^-64
}

// ---------------------------------------------------------------------------
// interpolation (node_pot, gqmap_gpu_mixture.m:157-176)
// ---------------------------------------------------------------------------
template <typename R>
GQ_HD void keys4(R t, R &w0, R &w1, R &w2, R &w3)
{
    // Keys a=-1/2 weights in the x2 form of the reference (they sum to 2):
    //   ((2-t)t-1)t, (3t-5)t^2+2, ((4-3t)t+1)t, (t-1)t^2
    // as 8 operations on t2 = t^2 and b = 4-3t (every constant an inline
    // operand or the one scalar -3):
    //   w0 = t2(2-t) - t,  w1 = (2-t2) - t2 b,  w2 = t2 b + t,  w3 = t2 t - t2
    const R t2 = t * t;
    const R b = fma(R(-3), t, R(4));
    w0 = fma(t2, R(2) - t, -t);
    w1 = fma(-t2, b, R(2) - t2);
    w2 = fma(t2, b, t);
    w3 = fma(t2, t, -t2);
}

#ifndef GQ_FRACT  // x - floor(x) (exact); the device has it as one instruction
#define GQ_FRACT(x) ((x) - floor(x))
#endif

#ifndef GQ_UMUL24  // 24-bit multiply (full rate on the device; both factors < 2^24)
#define GQ_UMUL24(a, b) ((uint32_t)(a) * (uint32_t)(b))
#endif

// Pointer `bytes` past the padded frame's base: a frame is < 4 GiB, so every
// gather is SGPR base + 32-bit VGPR offset (no 64-bit address arithmetic).
template <typename VP>
GQ_HD VP byte_ptr(VP VV, uint32_t bytes)
{
    return (VP)((const char *)VV + bytes);
}
template <typename VP>
GQ_HD VP elem_ptr(VP VV, uint32_t elem)
{
    return byte_ptr(VV, elem * (uint32_t)sizeof(*VV));
}

// Paired binary16 storage of the padded frame (policy vv_pair; the fp64
// single-scale mixture engine on frames whose padded values are all exact in
// binary16 -- the integer frames of rgb2gray, C2's within [-510, 765]):
// element (r, c) holds the values of columns c and c + 1 of row r, so one
// 16-byte load returns two tap columns of a cell and a sample needs two loads
// instead of four (the gathers' address work is what bounds the node loop
// beside the VALU: a timing probe with half the loads ran 14% faster).  Each
// tap converts exactly (binary16 -> float -> double): the same values, so the
// same bits as float or double storage.
#if defined(__HIPCC__)
struct alignas(4) vvh2_t {
    _Float16 lo, hi;  // columns c, c + 1
};
template <typename T>
struct is_vvh2 : std::is_same<typename std::remove_cv<T>::type, vvh2_t> {};
#else
template <typename T>
struct is_vvh2 : std::false_type {};
#endif
template <typename R, typename E>
GQ_HD R tap_col(const E &e, int half)
{
#if defined(__HIPCC__)
    if constexpr (is_vvh2<E>::value) return R((float)(half ? e.hi : e.lo));
    else
#endif
    {
        (void)half;
        return R(e);
    }
}

// 4 x the Keys interpolation (the reference's (sum of weighted taps)/4 before
// the /4): callers fold the 1/4 into their next operation, e.g. the residual
// I - v as fma(v4, -1/4, I) -- v4/4 is exact, so that is I - v bit for bit.
// o: element offset of the cell's first tap (top-left), M2: column stride.
template <typename R, typename VP>
GQ_HD R bicubic_w4(VP VV, uint32_t o, uint32_t M2, R s0, R s1, R s2, R s3, R t0, R t1, R t2, R t3)
{
    // taps are converted to R exactly (VV storage: double, or float when exact)
    constexpr uint32_t E = (uint32_t)sizeof(*VV);
    const uint32_t ob = o * E, cb = M2 * E;  // byte offsets: cell, column stride
    if constexpr (is_vvh2<typename std::remove_reference<decltype(*VV)>::type>::value) {
        const auto p0 = byte_ptr(VV, ob), p2 = byte_ptr(VV, ob + 2 * cb);  // columns 0, 1 / 2, 3
        R v[4];
        for (int c = 0; c < 4; ++c) {
            const auto p = c < 2 ? p0 : p2;
            const int h = c & 1;
            v[c] = fma(tap_col<R>(p[3], h), t3, fma(tap_col<R>(p[2], h), t2, fma(tap_col<R>(p[1], h), t1, tap_col<R>(p[0], h) * t0)));
        }
        return fma(s3, v[3], fma(s2, v[2], fma(s1, v[1], s0 * v[0])));
    } else {
        const auto c0 = byte_ptr(VV, ob);
        const R v0 = fma(R(c0[3]), t3, fma(R(c0[2]), t2, fma(R(c0[1]), t1, R(c0[0]) * t0)));
        const auto c1 = byte_ptr(VV, ob + cb);
        const R v1 = fma(R(c1[3]), t3, fma(R(c1[2]), t2, fma(R(c1[1]), t1, R(c1[0]) * t0)));
        const auto c2 = byte_ptr(VV, ob + 2 * cb);
        const R v2 = fma(R(c2[3]), t3, fma(R(c2[2]), t2, fma(R(c2[1]), t1, R(c2[0]) * t0)));
        const auto c3 = byte_ptr(VV, ob + 3 * cb);
        const R v3 = fma(R(c3[3]), t3, fma(R(c3[2]), t2, fma(R(c3[1]), t1, R(c3[0]) * t0)));
        return fma(s3, v3, fma(s2, v2, fma(s1, v1, s0 * v0)));
    }
}

// 4 x the Keys interpolation in the cell whose first tap is element o, at
// fraction so (columns) / to (rows).
template <typename R, typename VP>
GQ_HD R bicubic_cell4(VP VV, uint32_t o, uint32_t M2, R so, R to)
{
    R t0, t1, t2, t3, s0, s1, s2, s3;
    keys4(to, t0, t1, t2, t3);
    keys4(so, s0, s1, s2, s3);
    return bicubic_w4<R>(VV, o, M2, s0, s1, s2, s3, t0, t1, t2, t3);
}

// The same interpolation split in two, so a loop can issue the next sample's
// loads before this sample's arithmetic (node_sums, PF): the 16 taps of a
// cell in their storage type, then bicubic_w4's fma chain on them.
template <typename E>
struct Taps16 {
    E v[16];  // column-major: v[4 c + r], c columns from the cell's first tap
};
template <typename VP>
GQ_HD auto load_taps16(VP VV, uint32_t o, uint32_t M2)
{
    using E = typename std::remove_cv<typename std::remove_reference<decltype(*VV)>::type>::type;
    constexpr uint32_t EB = (uint32_t)sizeof(E);
    const uint32_t ob = o * EB, cb = M2 * EB;
    Taps16<E> T;
    if constexpr (is_vvh2<E>::value) {  // v[4 p + r]: row r of column pair p (columns 2p, 2p + 1)
        for (int pr = 0; pr < 2; ++pr) {
            const auto col = byte_ptr(VV, ob + (uint32_t)(2 * pr) * cb);
            for (int r = 0; r < 4; ++r) T.v[4 * pr + r] = col[r];
        }
        return T;
    } else {
        for (int c = 0; c < 4; ++c) {
            const auto col = byte_ptr(VV, ob + (uint32_t)c * cb);
            for (int r = 0; r < 4; ++r) T.v[4 * c + r] = col[r];
        }
        return T;
    }
}
template <typename R, typename E>
GQ_HD R bicubic_taps4(const Taps16<E> &T, R so, R to)
{
    R t0, t1, t2, t3, s0, s1, s2, s3;
    keys4(to, t0, t1, t2, t3);
    keys4(so, s0, s1, s2, s3);
    R v[4];
    if constexpr (is_vvh2<E>::value) {
        for (int c = 0; c < 4; ++c) {
            const E *p = T.v + 4 * (c >> 1);
            const int h = c & 1;
            v[c] = fma(tap_col<R>(p[3], h), t3, fma(tap_col<R>(p[2], h), t2, fma(tap_col<R>(p[1], h), t1, tap_col<R>(p[0], h) * t0)));
        }
    } else {
        for (int c = 0; c < 4; ++c)
            v[c] = fma(R(T.v[4 * c + 3]), t3, fma(R(T.v[4 * c + 2]), t2, fma(R(T.v[4 * c + 1]), t1, R(T.v[4 * c]) * t0)));
    }
    return fma(s3, v[3], fma(s2, v[2], fma(s1, v[1], s0 * v[0])));
}

GQ_HD uint32_t cell_elem(int iy, int ix, int M2) { return (uint32_t)(iy - 1) + GQ_UMUL24(M2, ix - 1); }

// Where the bicubic reads the padded frame: cell (iy, ix) (1-based) starts at
// element (iy - 1) + ld (ix - 1).  (Round 4 measured a per-tile LDS copy of
// the rectangle a tile's samples can reach, read through a windowed view of
// this kind: slower, profiles/r04_tap_lds_ab.txt -- not kept.)
template <typename VP>
struct TapView {
    VP p;
    uint32_t ld;
    GQ_HD uint32_t cell(int iy, int ix) const { return cell_elem(iy, ix, (int)ld); }
};
template <typename VP>
GQ_HD TapView<VP> frame_view(VP VV, int M2)
{
    return TapView<VP>{VV, (uint32_t)M2};
}

// Elements of a padded-frame (VV) buffer: the (Mo+2) x (No+2) frame, then
// zeros -- one column and a few elements (VV_TAIL, axis_cell_abs: the taps of
// cell (Mo, No) reach element (Mo+2) * (No+3)).
constexpr int VV_TAIL = 8;
constexpr size_t vv_elems(int Mo, int No) { return (size_t)(Mo + 2) * (size_t)(No + 3) + VV_TAIL; }

// One axis of sample()'s position arithmetic at the absolute 1-based
// position X on an axis of n pixels -> 1-based cell ix and fraction fr
// (fp64: the reference's own arithmetic: clamp to [1, n], floor).
//
// At X == n the reference's interp2 uses cell n-1 at fraction 1; here it is
// cell n at fraction 0 (no cap).  Both give the same value: the Keys weights
// are keys4(1) = (+0, +0, 2, +0) and keys4(0) = (+0, 2, +0, +0), so either
// fma chain is exactly 2 x the tap in column (row) n plus signed zeros from
// finite taps -- equal up to the sign of a zero result, which the residual
// I - v/4 and its square never see.  Cell n reads one tap past the padded
// frame (column No+2, row Mo+2): VV buffers carry a zero column and a few
// zero elements past the (Mo+2) x (No+2) frame (vv_elems).
template <bool CLAMP = true>
GQ_HD void axis_cell_abs(double X, int n, int &ix, double &fr)
{
    // min(max(.,1),N) with MATLAB's NaN-ignoring max/min (IEEE maxNum/minNum)
    if (CLAMP) X = fmin(fmax(X, 1.0), (double)n);
    ix = (int)X;       // X >= 1: truncation == floor
    fr = GQ_FRACT(X);  // X - floor(X)
}
// 1-based pixel j displaced by x (fp64: X = j + x, the reference's form).
template <bool CLAMP = true>
GQ_HD void axis_cell(int j, double x, int n, int &ix, double &fr)
{
    axis_cell_abs<CLAMP>((double)j + x, n, ix, fr);
}
// fp32: integer + fraction relative to the pixel, so the fractional position
// keeps full precision at any image size.
template <bool CLAMP = true>
GQ_HD void axis_cell(int j, float x, int n, int &ix, float &fr)
{
    if (CLAMP) x = fminf(fmaxf(x, (float)(1 - j)), (float)(n - j));
    const float f = floorf(x);
    fr = x - f;
    ix = j + (int)f;  // cell n at fraction 0 for x = n - j: see axis_cell_abs
}

// Relative form for both precisions: integer cell + fraction of the
// displacement x from the 1-based pixel j (the super engine's per-pixel path:
// an unclamped sample gets exactly the cell j + floor(x) and fraction
// x - floor(x) of the shared 7x7 window, so the two branches agree bit for bit).
template <typename R>
GQ_HD void axis_cell_rel(int j, R x, int n, int &ix, R &fr)
{
    x = fmin(fmax(x, R(1 - j)), R(n - j));
    const R f = floor(x);
    fr = x - f;
    ix = j + (int)f;
    if (ix > n - 1) { ix = n - 1; fr = R(1); }
}

// 4 x interp2-cubic at 1-based column jj + x1, row ii + x2 on the padded VV.
// CLAMP = false: the caller guarantees 1 <= jj + x1 < No and 1 <= ii + x2 < Mo
// for this sample, where every clamp is the identity -- same result.
// cell4_v: the cell's first tap and the fractions, sample4_v: the value.
template <bool CLAMP = true, typename TV, typename R>
GQ_HD uint32_t cell4_v(const TV &V, int Mo, int No, int ii, int jj, R x1, R x2, R &so, R &to)
{
    int ix, iy;
    axis_cell<CLAMP>(jj, x1, No, ix, so);
    axis_cell<CLAMP>(ii, x2, Mo, iy, to);
    return V.cell(iy, ix);
}
template <bool CLAMP = true, typename TV, typename R>
GQ_HD R sample4_v(const TV &V, int Mo, int No, int ii, int jj, R x1, R x2)
{
    R so, to;
    const uint32_t o = cell4_v<CLAMP>(V, Mo, No, ii, jj, x1, x2, so, to);
    return bicubic_cell4<R>(V.p, o, V.ld, so, to);
}
template <bool CLAMP = true, typename VP, typename R>
GQ_HD R sample4(VP VV, int M2, int Mo, int No, int ii, int jj, R x1, R x2)
{
    return sample4_v<CLAMP>(frame_view(VV, M2), Mo, No, ii, jj, x1, x2);
}
// fp64 at absolute 1-based positions X (column), Y (row).
template <bool CLAMP = true, typename TV>
GQ_HD uint32_t cell4_abs_v(const TV &V, int Mo, int No, double X, double Y, double &so, double &to)
{
    int ix, iy;
    axis_cell_abs<CLAMP>(X, No, ix, so);
    axis_cell_abs<CLAMP>(Y, Mo, iy, to);
    return V.cell(iy, ix);
}
template <bool CLAMP = true, typename TV>
GQ_HD double sample4_abs_v(const TV &V, int Mo, int No, double X, double Y)
{
    double so, to;
    const uint32_t o = cell4_abs_v<CLAMP>(V, Mo, No, X, Y, so, to);
    return bicubic_cell4<double>(V.p, o, V.ld, so, to);
}
template <bool CLAMP = true, typename VP>
GQ_HD double sample4_abs(VP VV, int M2, int Mo, int No, double X, double Y)
{
    return sample4_abs_v<CLAMP>(frame_view(VV, M2), Mo, No, X, Y);
}
// interp2-cubic itself (node_pot's Vq, gqmap_gpu_mixture.m:157-176).
template <bool CLAMP = true, typename VP, typename R>
GQ_HD R sample(VP VV, int M2, int Mo, int No, int ii, int jj, R x1, R x2)
{
    return sample4<CLAMP>(VV, M2, Mo, No, ii, jj, x1, x2) * R(0.25);
}

// Coarse-to-fine level data term (legacy/gqmap_ctf.m:10, 96):
//   I2_cont(clamp(round((m+x2-1)*64+1),1,MM), clamp(round((n+x1-1)*64+1),1,NN))
// with I2_cont = interp2(I2,6,'cubic') the 64x-refined cubic table.  A table
// entry (r, c) is the same Keys interpolation at (1+(c-1)/64, 1+(r-1)/64), so
// the lookup is sample() at the position rounded to the 1/64 grid -- the
// 64x table (10 GB at 480x640) is never built.  Returns 4 x the entry.
// max(round(y), 1) with MATLAB's round (half away from zero; NaN -> 1) as
// trunc(max(y, 1/2) + 1/2): for y >= 1/2 the sum y + 1/2 is exact or rounds
// within [2^k, 2^k + 1/2), so its truncation is floor(y + 1/2) = round(y);
// below 1/2 both give 1.  Four instructions instead of eight, same values.
template <typename R>
GQ_HD R round_ge1(R y)
{
    return trunc(fmax(y, R(0.5)) + R(0.5));
}

// CLAMP = false: the caller guarantees 1 <= jj + x1 < No - 1/64 (and the
// same for rows; node_unclamped with CTF_MARGIN), so round(y) lies in [1, MM)
// and no clamp or cap acts -- the same values.
template <bool CLAMP = true, typename TV, typename R>
GQ_HD uint32_t cell_ctf4_v(const TV &V, int Mo, int No, int ii, int jj, R x1, R x2, R &so, R &to)
{
    const R y = (((R)ii + x2) - R(1)) * R(64) + R(1), x = (((R)jj + x1) - R(1)) * R(64) + R(1);
    if constexpr (CLAMP) {
        const R MM = R(64 * (Mo - 1) + 1), NN = R(64 * (No - 1) + 1);
        const R ry = fmin(round_ge1(y), MM), rx = fmin(round_ge1(x), NN);
        const R Yq = (ry - R(1)) * R(0.015625) + R(1), Xq = (rx - R(1)) * R(0.015625) + R(1);
        int ix = (int)Xq, iy = (int)Yq;  // Xq in [1, No]: truncation == floor
        ix = ix > No - 1 ? No - 1 : ix;
        iy = iy > Mo - 1 ? Mo - 1 : iy;
        so = Xq - (R)ix;
        to = Yq - (R)iy;
        return V.cell(iy, ix);
    } else {
        const R ry = trunc(y + R(0.5)), rx = trunc(x + R(0.5));  // y, x >= 1: round_ge1
        const R Yq = (ry - R(1)) * R(0.015625) + R(1), Xq = (rx - R(1)) * R(0.015625) + R(1);
        const int ix = (int)Xq, iy = (int)Yq;
        so = GQ_FRACT(Xq);
        to = GQ_FRACT(Yq);
        return V.cell(iy, ix);
    }
}
template <bool CLAMP = true, typename TV, typename R>
GQ_HD R sample_ctf4_v(const TV &V, int Mo, int No, int ii, int jj, R x1, R x2)
{
    R so, to;
    const uint32_t o = cell_ctf4_v<CLAMP>(V, Mo, No, ii, jj, x1, x2, so, to);
    return bicubic_cell4<R>(V.p, o, V.ld, so, to);
}
template <bool CLAMP = true, typename VP, typename R>
GQ_HD R sample_ctf4(VP VV, int M2, int Mo, int No, int ii, int jj, R x1, R x2)
{
    return sample_ctf4_v<CLAMP>(frame_view(VV, M2), Mo, No, ii, jj, x1, x2);
}

// ---------------------------------------------------------------------------
// 4x4 super-pixel data term (gqmap_gpuSuper_mix_entropy.m:94-105):
//   sum_{i=top..bottom} sum_{j=left..right} sqrt(eps + (I1(i,j) - interp(j+x1, i+x2))^2)
// When no sample of the block is clamped (left+x1 >= 1, right+x1 <= No-1 and
// the same for rows) every sample has the fractional offset
// (so, to) = (x1 - floor(x1), x2 - floor(x2)) and pixel (i,j) interpolates the
// cell (i + floor(x2), j + floor(x1)): the 16 cells tile one 7x7 tap window,
// so the 28 column sums are shared (49 taps instead of 256).  Each output
// uses exactly the fma sequence of bicubic_cell.  Blocks touching the border
// take per-sample clamped positions (axis_cell_rel: the reference's clamp,
// relative to the pixel), which for an unclamped block give the same cells,
// fractions and bits as the shared window.
// I[q], q = 4*di + dj (j fastest, the reference loop order).
// ---------------------------------------------------------------------------
template <typename R, typename VP>
GQ_HD R super_block_sum(VP VV, int M2, int Mo, int No, int i0, int j0, R x1, R x2, R eps,
                        const R (&I)[16])
{
    // Both branches compute every output from the same cells, fractions and
    // fma sequence, so the choice never changes a result.
    const bool safe = R(j0 + 1) + x1 >= R(1) && R(j0 + 4) + x1 <= R(No - 1) && R(i0 + 1) + x2 >= R(1) &&
                      R(i0 + 4) + x2 <= R(Mo - 1);
    R f = 0;
    if (safe) {
        const R fx = floor(x1), fy = floor(x2);
        const R so = x1 - fx, to = x2 - fy;
        R t0, t1, t2, t3, s0, s1, s2, s3;
        keys4(to, t0, t1, t2, t3);
        keys4(so, s0, s1, s2, s3);
        // window origin: padded row i0 + fy, padded column j0 + fx (0-based)
        const uint32_t o = (uint32_t)(i0 + (int)fy) + (uint32_t)M2 * (uint32_t)(j0 + (int)fx);
        R out[4][4];
        GQ_UNROLL_FULL
        for (int a = 0; a < 7; ++a) {
            const auto c = elem_ptr(VV, o + (uint32_t)(a * M2));
            R v[4];
            GQ_UNROLL_FULL
            for (int di = 0; di < 4; ++di)
                v[di] = fma(R(c[di + 3]), t3, fma(R(c[di + 2]), t2, fma(R(c[di + 1]), t1, R(c[di]) * t0)));
            GQ_UNROLL_FULL
            for (int dj = 0; dj < 4; ++dj) {
                const int k = a - dj;  // this column is tap k of output column dj
                if (k < 0 || k > 3) continue;
                const R sk = k == 0 ? s0 : k == 1 ? s1 : k == 2 ? s2 : s3;
                GQ_UNROLL_FULL
                for (int di = 0; di < 4; ++di)
                    out[di][dj] = k == 0 ? sk * v[di] : fma(sk, v[di], out[di][dj]);
            }
        }
        for (int q = 0; q < 16; ++q) {
            const R d = fma(out[q >> 2][q & 3], R(-0.25), I[q]);  // I - out/4, bit for bit
            f = f + GQ_SQRT(fma(d, d, eps));
        }
    } else {
        // A block that some sample of crosses the border.  Rows: each
        // pixel row its own clamped cell and weights (axis_cell_rel: cell
        // i + floor(x2) unless it clamps -- <= 0: cell 1 at fraction 0,
        // >= Mo: cell Mo-1 at fraction 1 -- from one floor per axis).
        // Columns: the pixel columns whose cells j0+dj+1+floor(x1) do not
        // clamp share the window of seven tap columns of the safe branch --
        // per pixel row, each window column's row chain is computed once and
        // fed to the pixel columns that use it, in the fma order of
        // bicubic_w4.  A clamped pixel column has weights keys4(0) =
        // (+0, 2, +0, +0) at cell 1 or keys4(1) = (+0, +0, 2, +0) at cell
        // No-1, so its bicubic_w4 chain is exactly 2 x the row chain of tap
        // column 1 or No (up to the sign of an exact zero, which the residual
        // I - v/4 and its square never see).  Same values as sixteen
        // per-pixel bicubic_w4 calls with nine row chains per pixel row
        // instead of sixteen: C4 k_iter fp64 350 -> 300-327 us, fp32
        // 344-390 -> 288-322 us (profiles/r03_super_clamped.txt).
        const R fx = floor(x1), fy = floor(x2);
        const R sx = x1 - fx, sy = x2 - fy;
        const int ifx = (int)fx, ify = (int)fy;
        R s0, s1, s2, s3;
        keys4(sx, s0, s1, s2, s3);
        // pixel rows one at a time (few live registers), in the order of the
        // residual sum below (q = 4 di + dj)
        GQ_UNROLL_FULL
        for (int di = 0; di < 4; ++di) {
            const int r = i0 + di + 1 + ify;
            const int iy = r <= 0 ? 1 : r >= Mo ? Mo - 1 : r;
            R t0, t1, t2, t3;
            keys4(r <= 0 ? R(0) : r >= Mo ? R(1) : sy, t0, t1, t2, t3);
            const uint32_t rb = (uint32_t)(iy - 1);
            // the row chain of padded tap column col (bicubic_w4's v_a)
            auto chain = [&](int col) {
                const auto cp = elem_ptr(VV, rb + GQ_UMUL24(M2, col));
                return fma(R(cp[3]), t3, fma(R(cp[2]), t2, fma(R(cp[1]), t1, R(cp[0]) * t0)));
            };
            // branch-free: every window column is evaluated (its index kept
            // inside the padded frame; a column no unclamped pixel column
            // reads only feeds outputs that the clamped-column values below
            // replace), so divergent lanes run one straight-line body
            R o[4];
            GQ_UNROLL_FULL
            for (int a = 0; a < 7; ++a) {
                int col = j0 + ifx + a;
                col = col < 0 ? 0 : col > No + 1 ? No + 1 : col;
                const R v = chain(col);
                GQ_UNROLL_FULL
                for (int dj = 0; dj < 4; ++dj) {
                    const int k = a - dj;  // this column is tap k of pixel column dj
                    if (k < 0 || k > 3) continue;
                    const R sk = k == 0 ? s0 : k == 1 ? s1 : k == 2 ? s2 : s3;
                    o[dj] = k == 0 ? sk * v : fma(sk, v, o[dj]);
                }
            }
            const R vl = R(2) * chain(1), vr = R(2) * chain(No);  // padded tap columns 1 / No
            GQ_UNROLL_FULL
            for (int dj = 0; dj < 4; ++dj) {
                const int c = j0 + dj + 1 + ifx;
                o[dj] = c <= 0 ? vl : c >= No ? vr : o[dj];
            }
            GQ_UNROLL_FULL
            for (int dj = 0; dj < 4; ++dj) {
                const R d = fma(o[dj], R(-0.25), I[4 * di + dj]);
                f = f + GQ_SQRT(fma(d, d, eps));
            }
        }
    }
    return f;
}

// ---------------------------------------------------------------------------
// spectral quadrature of the node / edge potentials
// ---------------------------------------------------------------------------
template <typename R>
struct Grad {
    R da, du1, du2, do1, do2, dp, E;
};

// Basis sums: with f_k the potential at quadrature point k and table
// weights W_k = WIWJ(k),
//   s0 = sum W f, sxi = sum W XI f, sxj = sum W XJ f,
//   sa = sum W (XI^2+XJ^2) f, sm = sum W (XI^2-XJ^2) f, sx = sum W XI XJ f.
// Every accumulator of the reference (dp, du1, du2, do1, do2, Ei;
// gqmap_gpu_mixture.m:99-105) is a fixed linear combination of these six.
// Table rows: T_XI .. T_WX above.
template <typename R>
struct Sums {
    R s0 = 0, sxi = 0, sxj = 0, sa = 0, sm = 0, sx = 0;
    template <typename TP>
    GQ_HD void add(TP tab, int k, R f)
    {
        s0 = fma(tab[tab_at(T_W, k)], f, s0);
        sxi = fma(tab[tab_at(T_WXI, k)], f, sxi);
        sxj = fma(tab[tab_at(T_WXJ, k)], f, sxj);
        sa = fma(tab[tab_at(T_WA, k)], f, sa);
        sm = fma(tab[tab_at(T_WM, k)], f, sm);
        sx = fma(tab[tab_at(T_WX, k)], f, sx);
    }
    // point k and its mirror K^2-1-k (xi, xj -> -xi, -xj: the Gauss-Hermite
    // rule is symmetric, so w, w(xi^2+-xj^2), w xi xj are shared and w xi,
    // w xj change sign): fp = f(k), fm = f(mirror)
    template <typename TP>
    GQ_HD void add_pair(TP tab, int k, R fp, R fm)
    {
        const R fs = fp + fm, fd = fp - fm;
        s0 = fma(tab[tab_at(T_W, k)], fs, s0);
        sxi = fma(tab[tab_at(T_WXI, k)], fd, sxi);
        sxj = fma(tab[tab_at(T_WXJ, k)], fd, sxj);
        sa = fma(tab[tab_at(T_WA, k)], fs, sa);
        sm = fma(tab[tab_at(T_WM, k)], fs, sm);
        sx = fma(tab[tab_at(T_WX, k)], fs, sx);
    }
};

// Quadrature loop order shared by the node and edge sums.  The K x K
// points come in mirror pairs (k, K^2-1-k), k < K^2/2, plus the centre
// (k = (K^2-1)/2, xi = xj = 0) when K is odd.  Lane j of Q takes the pairs
// k = j, j+Q, ... in increasing k and, if (npairs - j) % Q == 0, the centre
// last.  body_pair(k) / body_center(k) do the evaluation and accumulation.
// PU: pairs per loop trip (0: the includer's GQ_PAIR_UNROLL; the order of
// the sums is the same for every PU).
template <int PU = 0, typename FP, typename FC>
GQ_HD void quad_pairs(int k0, int K2, int dk, FP body_pair, FC body_center)
{
    const int np = K2 >> 1;
    if constexpr (PU == 0) {
        GQ_PAIR_UNROLL
        for (int k = k0; k < np; k += dk) body_pair(k);
    } else {
        GQ_PAIR_UNROLL_K(PU)
        for (int k = k0; k < np; k += dk) body_pair(k);
    }
    if ((K2 & 1) && np >= k0 && (np - k0) % dk == 0) body_center(np);
}

template <typename R>
GQ_HD void spectral_st(R p, R &s, R &t)
{
    const R sp = GQ_SQRT(R(1) + p), sm = GQ_SQRT(R(1) - p);
    s = (sp + sm) * R(0.5);
    t = (sp - sm) * R(0.5);
}

// Epilogue shared by node (tau = -3T) and edge (tau = +T) gradients
// (gqmap_gpu_mixture.m:107-115 and :137-145).  lam = -lambda scales the sums.
//
// The reference divides by pi in six places; here 1/pi is folded into the
// sums' scale (lam/pi: one multiply per sum, six correctly rounded divisions
// fewer per node / edge gradient).  Each quotient differs from the
// reference's by a rounding or two (the literal restatement in oracle/ keeps
// the reference's order; the tests hold the two within 1e-12 per step).
// Replacing the remaining divisions by o1, o2, pr with reciprocals measured
// 13% slower on C2 fp64 (fp32 2% faster) and is not used.
template <typename R>
GQ_HD Grad<R> epilogue(const Sums<R> &S, R lam, R a, R o1, R o2, R p, R s, R t, R tau,
                       bool live, bool raw_energy = false)
{
    const R c1 = R(2.8378770664093454835606594728112);  // 1 + log(2*pi)
    const R lp = lam * R(1.0 / GQ_M_PI);
    const R S0 = lp * S.s0, Sxi = lp * S.sxi, Sxj = lp * S.sxj;
    const R Sa = lp * S.sa, Sm = lp * S.sm, Sx = lp * S.sx;
    const R pr = R(1) - p * p;
    const R sqrtpr = GQ_SQRT(pr);
    const R a1 = s - p * t, a2 = t - p * s;
    R dp = p * (S0 - Sa) + R(2) * Sx;
    R du1 = a1 * Sxi + a2 * Sxj;
    R du2 = a2 * Sxi + a1 * Sxj;
    const R smr = Sm / sqrtpr;
    R do1 = (Sa - S0) + smr;
    R do2 = (Sa - S0) - smr;
    if (!live) dp = du1 = du2 = do1 = do2 = R(0);
    Grad<R> g;
    const R sq2 = R(GQ_M_SQRT2);
    g.du1 = a * du1 * (sq2 / (o1 * pr));
    g.du2 = a * du2 * (sq2 / (o2 * pr));
    const R ent = tau != R(0) ? tau * (c1 + gq_logr<R>(sqrtpr * o1 * o2)) : R(0);
    g.da = S0 + ent;
    g.do1 = a * (do1 + tau) / o1;
    g.do2 = a * (do2 + tau) / o2;
    g.dp = a * (dp - tau * p) / pr;
    // gqmap_ctf.m's nener/eener = -lambda*sum(fval): no 1/pi, no alpha
    g.E = raw_energy ? lam * S.s0 : a * g.da;
    return g;
}

// Sums over a split quadrature: lane j of Q accumulates k = j, j+Q, ... in
// increasing k; the Q partial sums are combined by an xor butterfly
// (offsets Q/2, ..., 1): total = ((p0+p_{Q/2}) + ...) -- butterfly() below is
// the reference evaluation of that order, the kernel does it with shuffles.
template <typename R>
GQ_HD Sums<R> sums_plus(const Sums<R> &a, const Sums<R> &b)
{
    Sums<R> r;
    r.s0 = a.s0 + b.s0; r.sxi = a.sxi + b.sxi; r.sxj = a.sxj + b.sxj;
    r.sa = a.sa + b.sa; r.sm = a.sm + b.sm; r.sx = a.sx + b.sx;
    return r;
}
// Q = 64 is the one-wave-per-node form of the smallest grids: the node's
// quadrature over the 64 lanes of its wave, each edge over a 16-lane group
// (edge_parts).
constexpr int edge_parts(int Q) { return Q > 16 ? 16 : Q; }
template <typename R>
GQ_HD Sums<R> butterfly(const Sums<R> *parts, int Q)
{
    Sums<R> v[64];
    for (int j = 0; j < Q; ++j) v[j] = parts[j];
    for (int o = Q / 2; o > 0; o >>= 1) {
        Sums<R> w[64];
        for (int j = 0; j < Q; ++j) w[j] = sums_plus(v[j], v[j ^ o]);
        for (int j = 0; j < Q; ++j) v[j] = w[j];
    }
    return v[0];
}

// edge_grad_spectral (gqmap_gpu_mixture.m:118-146) with edge_pot (:180-182):
// x1 - x2 = sqrt2*o1*(s XI + t XJ) + u1 - sqrt2*o2*(t XI + s XJ) - u2
template <typename R>
struct EdgeCoef {
    R s, t, A, B, C;
};
template <typename R>
GQ_HD EdgeCoef<R> edge_coef(R u1, R u2, R o1, R o2, R p)
{
    EdgeCoef<R> c;
    spectral_st(p, c.s, c.t);
    const R sq2 = R(GQ_M_SQRT2);
    c.A = sq2 * (o1 * c.s - o2 * c.t);
    c.B = sq2 * (o1 * c.t - o2 * c.s);
    c.C = u1 - u2;
    return c;
}
template <int PU = 0, typename R, typename TP>
GQ_HD Sums<R> edge_sums(TP tab, int k0, int K2, int dk, R eps, const EdgeCoef<R> &c)
{
    Sums<R> S;
    quad_pairs<PU>(
        k0, K2, dk,
        [&](int k) {
            // d = C +- p with p = A xi + B xj
            const R p = fma(c.A, tab[tab_at(T_XI, k)], c.B * tab[tab_at(T_XJ, k)]);
            const R dp = c.C + p, dm = c.C - p;
            S.add_pair(tab, k, GQ_SQRT(fma(dp, dp, eps)), GQ_SQRT(fma(dm, dm, eps)));
        },
        [&](int k) {
            const R d = fma(c.A, tab[tab_at(T_XI, k)], fma(c.B, tab[tab_at(T_XJ, k)], c.C));
            S.add(tab, k, GQ_SQRT(fma(d, d, eps)));
        });
    return S;
}
template <typename R>
GQ_HD Grad<R> edge_epi(const Sums<R> &S, const EdgeCoef<R> &c, R lams, bool guard, R T, R a, R o1,
                       R o2, R p, bool raw_energy = false)
{
    return epilogue(S, -lams, a, o1, o2, p, c.s, c.t, T, !guard || a != R(0), raw_energy);
}
template <typename R, typename TP>
GQ_HD Grad<R> edge_grad(TP tab, int K2, R eps, R lams, bool guard, R T, R a, R u1, R u2, R o1,
                        R o2, R p)
{
    const EdgeCoef<R> c = edge_coef(u1, u2, o1, o2, p);
    return edge_epi(edge_sums(tab, 0, K2, 1, eps, c), c, lams, guard, T, a, o1, o2, p);
}

// node_grad_spectral (gqmap_gpu_mixture.m:87-116; super: gqmap_gpuSuper_mix_entropy.m:87-122).
// (m, n) 0-based node; single-scale reads pixel (m, n), super the 4x4 block.
template <typename R>
struct NodeCoef {
    R s, t, ax, bx, ay, by;  // x1 = ax XI + bx XJ + u1, x2 = ay XI + by XJ + u2
};
template <typename R>
GQ_HD NodeCoef<R> node_coef(R o1, R o2, R p)
{
    NodeCoef<R> c;
    spectral_st(p, c.s, c.t);
    const R sq2 = R(GQ_M_SQRT2);
    c.ax = sq2 * o1 * c.s; c.bx = sq2 * o1 * c.t;
    c.ay = sq2 * o2 * c.t; c.by = sq2 * o2 * c.s;
    return c;
}
// ENG: 0 single-scale mixture, 1 super (4x4 blocks), 2 coarse-to-fine level.
// CLAMP = false (ENG 0): the caller has checked that no sample of this node
// is clamped (node_unclamped), so the clamps are skipped -- same results.
// V: where the taps are read (TapView: the frame, or the single-pixel
// engines' staged window).
// PF: software-pipelined -- sample k + dk's cell is located and its 16 taps
// loaded before sample k's arithmetic, so the gather latency overlaps it
// (the small-grid kernels run 1-2 waves per SIMD, memory waits dominating);
// the same operations on the same operands, so the same bits.
template <int ENG, bool CLAMP = true, bool PF = false, typename R, typename TP, typename TV, typename IP>
GQ_HD Sums<R> node_sums(TP tab, int k0, int K2, int dk, const TV &V, IP I1, int Mo, int No,
                        R eps, const NodeCoef<R> &c, R u1, R u2, int m, int n)
{
    Sums<R> S;
    if constexpr (PF && ENG != 1) {
        const R I = I1[m + (int64_t)Mo * n];
        constexpr bool ABS = ENG == 0 && sizeof(R) == 8;
        const R U1 = ABS ? u1 + R(n + 1) : u1, U2 = ABS ? u2 + R(m + 1) : u2;
        // cell and fractions of sample k
        auto locate = [&](int k, R &so, R &to) -> uint32_t {
            const R x1 = fma(c.ax, tab[tab_at(T_XI, k)], fma(c.bx, tab[tab_at(T_XJ, k)], U1));
            const R x2 = fma(c.ay, tab[tab_at(T_XI, k)], fma(c.by, tab[tab_at(T_XJ, k)], U2));
            if constexpr (ABS) return cell4_abs_v<CLAMP>(V, Mo, No, (double)x1, (double)x2, so, to);
            else if constexpr (ENG == 2) return cell_ctf4_v<CLAMP>(V, Mo, No, m + 1, n + 1, x1, x2, so, to);
            else return cell4_v<CLAMP>(V, Mo, No, m + 1, n + 1, x1, x2, so, to);
        };
        if (k0 < K2) {
            const int klast = k0 + (K2 - 1 - k0) / dk * dk;
            R so, to;
            auto T = load_taps16(V.p, locate(k0, so, to), V.ld);
            for (int k = k0; k <= klast; k += dk) {
                const auto Tk = T;
                const R sok = so, tok = to;
                const int kn = k + dk <= klast ? k + dk : klast;  // the last pass reloads its own cell
                T = load_taps16(V.p, locate(kn, so, to), V.ld);
                const R d = fma(bicubic_taps4<R>(Tk, sok, tok), R(-0.25), I);
                S.add(tab, k, GQ_SQRT(fma(d, d, eps)));
            }
        }
        return S;
    }
    if constexpr (ENG != 1) {
        const R I = I1[m + (int64_t)Mo * n];
        if constexpr (ENG == 0 && sizeof(R) == 8) {
            // fp64 single-scale: absolute positions X = j + x1 with the pixel
            // folded into the mean once per node (U1 = u1 + j)
            const R U1 = u1 + R(n + 1), U2 = u2 + R(m + 1);
            GQ_NODE_UNROLL
            for (int k = k0; k < K2; k += dk) {
                const R X = fma(c.ax, tab[tab_at(T_XI, k)], fma(c.bx, tab[tab_at(T_XJ, k)], U1));
                const R Y = fma(c.ay, tab[tab_at(T_XI, k)], fma(c.by, tab[tab_at(T_XJ, k)], U2));
                const R d = fma(sample4_abs_v<CLAMP>(V, Mo, No, X, Y), R(-0.25), I);
                S.add(tab, k, GQ_SQRT(fma(d, d, eps)));
            }
        } else {
            // one point at a time in increasing k (mirror pairs sample far-apart
            // cells: measured slower for the gathers, unlike the edge sums)
            GQ_NODE_UNROLL
            for (int k = k0; k < K2; k += dk) {
                const R x1 = fma(c.ax, tab[tab_at(T_XI, k)], fma(c.bx, tab[tab_at(T_XJ, k)], u1));
                const R x2 = fma(c.ay, tab[tab_at(T_XI, k)], fma(c.by, tab[tab_at(T_XJ, k)], u2));
                const R v4 = ENG == 2 ? sample_ctf4_v<CLAMP>(V, Mo, No, m + 1, n + 1, x1, x2)
                                      : sample4_v<CLAMP>(V, Mo, No, m + 1, n + 1, x1, x2);
                const R d = fma(v4, R(-0.25), I);
                S.add(tab, k, GQ_SQRT(fma(d, d, eps)));
            }
        }
    } else {
        // super = sum_{i=top..bottom} sum_{j=left..right} node_pot(x1,x2,i,j): j fastest
        R I[16];
        const int i0 = 4 * m, j0 = 4 * n;  // 0-based top-left pixel of the block
        for (int q = 0; q < 16; ++q) I[q] = I1[(i0 + (q >> 2)) + (int64_t)Mo * (j0 + (q & 3))];
        // (one point at a time: a pair of 4x4 block sums costs more VGPRs than it saves)
        for (int k = k0; k < K2; k += dk) {
            const R x1 = fma(c.ax, tab[tab_at(T_XI, k)], fma(c.bx, tab[tab_at(T_XJ, k)], u1));
            const R x2 = fma(c.ay, tab[tab_at(T_XI, k)], fma(c.by, tab[tab_at(T_XJ, k)], u2));
            S.add(tab, k, super_block_sum<R>(V.p, (int)V.ld, Mo, No, i0, j0, x1, x2, eps, I));
        }
    }
    return S;
}
// Conservative test that every quadrature sample of node (m, n) (0-based)
// lies where sample()'s clamps are the identity: |x1 - u1| <= (|ax|+|bx|) xmax
// and |x2 - u2| <= (|ay|+|by|) xmax (xmax = max |Gauss-Hermite node|), with a
// margin far above the rounding of the position arithmetic.
// (ctf engine: extra = CTF_MARGIN, the 1/64-grid rounding of the position
// must not reach the last column / row either)
constexpr double CTF_MARGIN = 1.0 / 32;
template <typename R>
GQ_HD bool node_unclamped(const NodeCoef<R> &c, R u1, R u2, int m, int n, int Mo, int No, R xmax, R extra = R(0))
{
    const R margin = (sizeof(R) == 8 ? R(1e-6) : R(1e-2)) + extra;
    const R rx = (fabs(c.ax) + fabs(c.bx)) * xmax + margin, ry = (fabs(c.ay) + fabs(c.by)) * xmax + margin;
    // positions relative to the 1-based pixel (n+1, m+1)
    return u1 - rx >= R(-n) && u1 + rx < R(No - 1 - n) && u2 - ry >= R(-m) && u2 + ry < R(Mo - 1 - m);
}

template <typename R>
GQ_HD Grad<R> node_epi(const Sums<R> &S, const NodeCoef<R> &c, R lamd, bool guard, R T, R a, R o1,
                       R o2, R p, bool raw_energy = false)
{
    return epilogue(S, -lamd, a, o1, o2, p, c.s, c.t, R(-3) * T, !guard || a != R(0), raw_energy);
}
template <int ENG, typename R, typename TP, typename VP, typename IP>
GQ_HD Grad<R> node_grad(TP tab, int K2, VP VV, IP I1, int M2, int Mo, int No, R eps, R lamd,
                        bool guard, R T, R a, R u1, R u2, R o1, R o2, R p, int m, int n)
{
    const NodeCoef<R> c = node_coef(o1, o2, p);
    return node_epi(node_sums<ENG>(tab, 0, K2, 1, frame_view(VV, M2), I1, Mo, No, eps, c, u1, u2, m, n), c,
                    lamd, guard, T, a, o1, o2, p, ENG == 2);
}

// ---------------------------------------------------------------------------
// Literal-order arithmetic (gqmap_options.arith = GQMAP_ARITH_LITERAL; fp64,
// single-scale mixture engine, one lane per node).
//
// The fast specification above regroups the reference's arithmetic (basis
// sums, fma, 1/pi folded into a scale, absolute sample positions, mirror
// pairs): each gradient differs from the reference's by a rounding or two.
// This variant evaluates every expression of node_grad_spectral /
// edge_grad_spectral / node_pot / edge_pot (gqmap_gpu_mixture.m:87-182) in
// MATLAB's left-to-right order with no fused operation: products of three
// as (a*b)*c, the K^2 quadrature points summed one after the other in
// meshgrid order, XI2mXJ2(k)/sqrtpr divided per point, the six divisions by
// pi where the reference has them.  With L = 1 and T = 0 (config C2) every
// operation of an iteration is then a correctly rounded IEEE +, -, *, /,
// sqrt, floor or min/max on the same operands as oracle/gqmap_oracle.c
// (compiled -ffp-contract=off), so the two agree bit for bit at any
// iteration count (tests/test_emulator.py, tests/test_gpu_literal.py) given
// the same Gauss-Hermite rule.  (T != 0 adds the entropy log, here the
// deterministic gq_log instead of libm's log.)  The exact fixed-point pixel
// sums (Energy, ptdmu) are not part of the state update; they are the
// correctly rounded sums of the reference's summands.
//
// Table rows of a quadrature point in this mode (the 8-entry point-major
// layout of tab_at): XI, XJ, WIWJ, XI2aXJ2, XI2mXJ2, 2*XIXJ (exact
// doubling), XI2aXJ2 - 1 (the reference's per-point value: same rounding
// whether it is formed here or in the loop), unused.
// ---------------------------------------------------------------------------
constexpr int TL_XI = 0, TL_XJ = 1, TL_W = 2, TL_A = 3, TL_M = 4, TL_X2 = 5, TL_A1 = 6;

// gqmap_gpu_mixture.m:8-10 (meshgrid: XI(r,c) = X(c), XJ(r,c) = X(r)) for one
// point k = r + K c: row8 receives the 8 table entries above.  (Host code:
// gqmap_create builds the table.)
#ifdef __HIPCC__
__host__ __device__
#endif
inline void lit_table_point(double *row8, double xi, double xj, double wi, double wj)
{
    const double a = xi * xi + xj * xj;
    row8[TL_XI] = xi;
    row8[TL_XJ] = xj;
    row8[TL_W] = wi * wj;
    row8[TL_A] = a;
    row8[TL_M] = xi * xi - xj * xj;
    row8[TL_X2] = 2 * (xi * xj);
    row8[TL_A1] = a - 1;
    row8[7] = 0;
}

// node_pot's interpolation (gqmap_gpu_mixture.m:157-176) in its own order:
// Xq, Yq clamped to [1, N] x [1, M], the cell chosen by the reference's
// if-chain, each tap weighted as (VV * ss) * tw, the taps added left to right
// (first column parenthesised as the reference writes it), then /4.
//
// Execution forms of the literal loops (GQ_LIT_FORM; every form performs the
// same IEEE operations on the same operands, so the bits never change --
// tests/test_literal.py, tests/test_gpu_literal.py):
//   0  round 5: the reference's if-chain as branches, `if a~=0` per point,
//      every product of a point formed at the point;
//   1  the cell chosen branch-free: after the clamp Xq is in [1, N], where
//      the chain's 1 / floor(Xq) / N-1 is exactly min(floor(Xq), N-1) (the
//      chain's first arm only sees Xq = 1 = floor(Xq)); `a~=0` is uniform
//      over a gradient (alpha of one component, one guard flag), so the
//      loop is versioned on it instead of testing it per point;
//   2  as 1, and the column's products s*XI, t*XI formed once per meshgrid
//      column (XI(r, c) = X(c) for every row r, gqmap_gpu_mixture.m:8): the
//      same rounded products the per-point form computes.
#ifndef GQ_LIT_FORM
#define GQ_LIT_FORM 2
#endif
// the three changes separately (A/B): branch-free cell, versioned loop,
// column products (default: those of GQ_LIT_FORM)
#ifndef GQ_LIT_CELL
#define GQ_LIT_CELL (GQ_LIT_FORM >= 1)
#endif
#ifndef GQ_LIT_HOIST
#define GQ_LIT_HOIST (GQ_LIT_FORM >= 1)
#endif
#ifndef GQ_LIT_CSE
#define GQ_LIT_CSE (GQ_LIT_FORM >= 2)
#endif
// fmin / fmax of non-NaN operands (the clamp's): on the device the bare
// v_min_f64 / v_max_f64.  Through fmin the compiler re-canonicalises the
// loop-invariant bound (a v_max_f64 x, x) at every quadrature point -- 4 of
// the node loop's ~174 VALU instructions.  The same IEEE result: min / max of
// two numbers is exact, and a NaN operand gives the other one either way.
GQ_HD double lit_min(double a, double b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return fmin(a, b);
#endif
}
GQ_HD double lit_max(double a, double b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return fmax(a, b);
#endif
}
#ifndef GQ_LIT_ASM_MINMAX
#define GQ_LIT_ASM_MINMAX 1
#endif
#if GQ_LIT_ASM_MINMAX
#define GQ_LMIN lit_min
#define GQ_LMAX lit_max
#else
#define GQ_LMIN fmin
#define GQ_LMAX fmax
#endif
// GQ_LIT_ADDR: the four tap columns as one cell offset plus multiples of the
// column stride (byte offsets, as bicubic_w4) instead of a multiply each.
// With GQ_LIT_ASM_MINMAX: 174 -> 165 VALU instructions per node-gradient
// point, k_iter_lit 271.8 -> 268.1 us, graph 255.0 -> 250.4 us per iteration,
// the same checksum (profiles/r06_lit_minmax_addr_ab.txt).
#ifndef GQ_LIT_ADDR
#define GQ_LIT_ADDR 1
#endif
template <typename VP>
GQ_HD double lit_interp(VP VV, int M2, int Mo, int No, double Xq, double Yq)
{
    Xq = GQ_LMIN(GQ_LMAX(Xq, 1.0), (double)No);
    Yq = GQ_LMIN(GQ_LMAX(Yq, 1.0), (double)Mo);
#if GQ_LIT_CELL
    const double fx = GQ_LMIN(floor(Xq), (double)(No - 1)), fy = GQ_LMIN(floor(Yq), (double)(Mo - 1));
    const int ix = (int)fx, iy = (int)fy;
    const double so = Xq - fx, to = Yq - fy;
#else
    int ix, iy;
    if (Xq <= 1.0) ix = 1;
    else if (Xq <= No - 1) ix = (int)floor(Xq);
    else ix = No - 1;
    if (Yq <= 1.0) iy = 1;
    else if (Yq <= Mo - 1) iy = (int)floor(Yq);
    else iy = Mo - 1;
    const double so = Xq - ix, to = Yq - iy;
#endif
    const double t0 = ((2.0 - to) * to - 1.0) * to;
    const double t1 = (3.0 * to - 5.0) * to * to + 2.0;
    const double t2 = ((4.0 - 3.0 * to) * to + 1.0) * to;
    const double t3 = (to - 1.0) * to * to;
#if GQ_LIT_ADDR
    constexpr uint32_t E = (uint32_t)sizeof(*VV);
    const uint32_t ob = cell_elem(iy, ix, M2) * E, cb = (uint32_t)M2 * E;
    const auto c1 = byte_ptr(VV, ob);
    const auto c2 = byte_ptr(VV, ob + cb);
    const auto c3 = byte_ptr(VV, ob + 2 * cb);
    const auto c4 = byte_ptr(VV, ob + 3 * cb);
#else
    const auto c1 = elem_ptr(VV, cell_elem(iy, ix, M2));
    const auto c2 = elem_ptr(VV, cell_elem(iy, ix + 1, M2));
    const auto c3 = elem_ptr(VV, cell_elem(iy, ix + 2, M2));
    const auto c4 = elem_ptr(VV, cell_elem(iy, ix + 3, M2));
#endif
    double ss = ((2.0 - so) * so - 1.0) * so;
    double Vq = (((double)c1[0] * ss * t0 + (double)c1[1] * ss * t1) + (double)c1[2] * ss * t2) +
                (double)c1[3] * ss * t3;
    ss = (3.0 * so - 5.0) * so * so + 2.0;
    Vq = Vq + (double)c2[0] * ss * t0 + (double)c2[1] * ss * t1 + (double)c2[2] * ss * t2 + (double)c2[3] * ss * t3;
    ss = ((4.0 - 3.0 * so) * so + 1.0) * so;
    Vq = Vq + (double)c3[0] * ss * t0 + (double)c3[1] * ss * t1 + (double)c3[2] * ss * t2 + (double)c3[3] * ss * t3;
    ss = (so - 1.0) * so * so;
    Vq = Vq + (double)c4[0] * ss * t0 + (double)c4[1] * ss * t1 + (double)c4[2] * ss * t2 + (double)c4[3] * ss * t3;
    return Vq / 4;
}

// x / y correctly rounded, given yr = RN(1 / y) (GQ_LIT_MDIV, device only):
// q0 = RN(x yr) is within 1.5 ulp of x / y, one correction
// RN(q0 + RN(x - y q0) yr) brings it within 1 ulp, and a second is RN(x / y)
// exactly (Markstein's theorem: yr within half an ulp of 1 / y, q within one
// ulp of x / y; no overflow or underflow for these operands: |x| < 64 and
// sqrtpr >= sqrt(1 - corr_tor^2) > 0, |p| <= corr_tor < 1) -- 5 operations
// instead of the 12 of the general IEEE sequence; the host divides.  Round 5
// (profiles/r05_literal_div_ab.txt): the literal engine's k_iter 327 -> 298 us
// on C2, still bit-identical to the restatement over 500 iterations.
#ifndef GQ_LIT_MDIV
#define GQ_LIT_MDIV 1
#endif
GQ_HD double div_rcp(double x, double y, double yr)
{
#if GQ_LIT_MDIV && defined(__HIP_DEVICE_COMPILE__)
    double q = x * yr;
    q = fma(fma(-q, y, x), yr, q);
    return fma(fma(-q, y, x), yr, q);
#else
    (void)yr;
    return x / y;
#endif
}

// The six accumulators of the quadrature loop (gqmap_gpu_mixture.m:98-105)
struct LitAcc {
    double dp = 0, du1 = 0, du2 = 0, do1 = 0, do2 = 0, Ei = 0;
    template <typename TP>
    GQ_HD void add(TP tab, int k, double fval, double zi, double zj, double p, double sqrtpr, double rsqrtpr,
                   bool live)
    {
        if (live) {  // `if a~=0` (:98)
            dp = dp + fval * ((p - p * tab[tab_at(TL_A, k)]) + tab[tab_at(TL_X2, k)]);
            du1 = du1 + fval * (zi - p * zj);
            du2 = du2 + fval * (zj - p * zi);
            const double q = div_rcp(tab[tab_at(TL_M, k)], sqrtpr, rsqrtpr);
            do1 = do1 + fval * (tab[tab_at(TL_A1, k)] + q);
            do2 = do2 + fval * (tab[tab_at(TL_A1, k)] - q);
        }
        Ei = Ei + fval;
    }
};

// K of a K x K rule from K2 (uniform, a few scalar steps)
GQ_HD int lit_k(int K2)
{
    int K = 1;
    while (K * K < K2) ++K;
    return K;
}

// Spectral coordinates shared by both gradients (:90-93, :120-123)
struct LitCoef {
    double s, t, pr, sqrtpr, rsqrtpr;  // rsqrtpr = RN(1 / sqrtpr) (div_rcp)
};
GQ_HD LitCoef lit_coef(double p)
{
    LitCoef c;
    const double sp = GQ_SQRT(1 + p), sm = GQ_SQRT(1 - p);
    c.s = (sp + sm) / 2;
    c.t = (sp - sm) / 2;
    c.pr = 1 - p * p;
    c.sqrtpr = GQ_SQRT(c.pr);
    c.rsqrtpr = 1 / c.sqrtpr;
    return c;
}

// Epilogues: node (:107-115, entropy -3T) and edge (:137-145, entropy +T).
// GQ_LIT_PIDIV: the six divisions by pi as div_rcp with RN(1/pi) (5
// operations instead of the general division's ~10; the same correctly
// rounded quotient -- div_rcp's conditions hold: pi's reciprocal rounded
// once, sums far from overflow and underflow).  Bit-identical over
// tests/test_gpu_literal.py, but neutral (264.9 vs 263.7 us, 30 of ~32k
// instructions per node-lane; profiles/r06_lit_xj_pidiv_ab.txt): off.
#ifndef GQ_LIT_PIDIV
#define GQ_LIT_PIDIV 0
#endif
GQ_HD double lit_div_pi(double x)
{
#if GQ_LIT_PIDIV
    constexpr double rpi = 1.0 / GQ_M_PI;
    return div_rcp(x, GQ_M_PI, rpi);
#else
    return x / GQ_M_PI;
#endif
}
GQ_HD Grad<double> lit_epi(const LitAcc &S, const LitCoef &c, double a, double o1, double o2, double p, double T,
                           bool node)
{
    const double o1pr = GQ_M_SQRT2 / (o1 * c.pr), o2pr = GQ_M_SQRT2 / (o2 * c.pr);
    Grad<double> g;
    g.du1 = lit_div_pi(a * S.du1 * o1pr);
    g.du2 = lit_div_pi(a * S.du2 * o2pr);
    // T (const1 + log(.)): a finite value times 0 when T = 0 -- skipped then
    // (the difference Ei/pi -+ 0 is Ei/pi: Ei < 0 never vanishes)
    const double ent = T != 0 ? (1 + gq_log(2 * GQ_M_PI)) + gq_log(c.sqrtpr * o1 * o2) : 0.0;
    if (node) {
        g.da = lit_div_pi(S.Ei) - 3 * T * ent;
        g.do1 = a * (lit_div_pi(S.do1) - 3 * T) / o1;
        g.do2 = a * (lit_div_pi(S.do2) - 3 * T) / o2;
        g.dp = a * (lit_div_pi(S.dp) + 3 * T * p) / c.pr;
    } else {
        g.da = lit_div_pi(S.Ei) + T * ent;
        g.do1 = a * (lit_div_pi(S.do1) + T) / o1;
        g.do2 = a * (lit_div_pi(S.do2) + T) / o2;
        g.dp = a * (lit_div_pi(S.dp) - T * p) / c.pr;
    }
    g.E = a * g.da;
    return g;
}

// The quadrature loop of a gradient, points k = r + K c in meshgrid order
// (column c outer, row r inner: the reference's k = 1..K^2): pt(k, zi, zj)
// returns the point's fval.  Form 2 forms s*XI and t*XI once per column.
// GQ_LIT_XJ_PREFETCH: the next point's XJ (a scalar load) issued during
// this point, so a point does not start with a wait on the scalar cache.
// Measured 263.7 -> 298.3 us (the node loop's schedule falls apart, as with
// GQ_LIT_NODE_UNROLL; profiles/r06_lit_xj_pidiv_ab.txt): off.
#ifndef GQ_LIT_XJ_PREFETCH
#define GQ_LIT_XJ_PREFETCH 0
#endif
template <bool LIVE, typename TP, typename PT>
GQ_HD void lit_points(TP tab, int K2, const LitCoef &c, double p, LitAcc &S, PT pt)
{
#if GQ_LIT_CSE
    const int K = lit_k(K2);
#if GQ_LIT_XJ_PREFETCH
    double XJn = tab[tab_at(TL_XJ, 0)];
#endif
    for (int cc = 0, k = 0; cc < K; ++cc) {
        const double XI = tab[tab_at(TL_XI, k)];
        const double sXI = c.s * XI, tXI = c.t * XI;
        for (int r = 0; r < K; ++r, ++k) {
#if GQ_LIT_XJ_PREFETCH
            const double XJ = XJn;
            XJn = tab[tab_at(TL_XJ, k + 1 < K2 ? k + 1 : k)];
#else
            const double XJ = tab[tab_at(TL_XJ, k)];
#endif
            const double zi = sXI + c.t * XJ, zj = tXI + c.s * XJ;
            S.add(tab, k, pt(k, zi, zj), zi, zj, p, c.sqrtpr, c.rsqrtpr, LIVE);
        }
    }
#else
    for (int k = 0; k < K2; ++k) {
        const double XI = tab[tab_at(TL_XI, k)], XJ = tab[tab_at(TL_XJ, k)];
        const double zi = c.s * XI + c.t * XJ, zj = c.t * XI + c.s * XJ;
        S.add(tab, k, pt(k, zi, zj), zi, zj, p, c.sqrtpr, c.rsqrtpr, LIVE);
    }
#endif
}

// Form 3 (GQ_LIT_MIRROR, edge gradients at K = 9): rows r and K-1-r of a
// meshgrid column share A = XI^2+XJ^2, M = XI^2-XJ^2 and A - 1 exactly (the
// library's Gauss-Hermite rule is symmetric: x(K-1-i) = -x(i), the middle
// node 0 -- gauss_hermite), so the same p - p*A, the same division M/sqrtpr
// and the same do-factors; XJ and 2*XI*XJ only flip sign.  The later row
// reuses the earlier row's rounded values instead of recomputing them: the
// same operations on the same operands as the per-point form, in the same
// accumulation order.  The column's pending values live in registers (the
// column loop fully unrolled).
#ifndef GQ_LIT_MIRROR
#define GQ_LIT_MIRROR 1
#endif
#ifndef GQ_LIT_MIRROR_NODE  // the same sharing in the node gradient's loop
#define GQ_LIT_MIRROR_NODE 0
#endif
template <int KK, typename TP, typename PT>
GQ_HD void lit_points_mirror(TP tab, const LitCoef &c, double p, LitAcc &S, PT pt)
{
    constexpr int H = KK / 2;
    for (int cc = 0, k0 = 0; cc < KK; ++cc, k0 += KK) {
        const double XI = tab[tab_at(TL_XI, k0)];
        const double sXI = c.s * XI, tXI = c.t * XI;
        double pA[H], F1[H], F2[H];
#ifdef __HIPCC__
#pragma unroll
#endif
        for (int r = 0; r < KK; ++r) {
            const int k = k0 + r;
            const double XJ = tab[tab_at(TL_XJ, k)];
            const double zi = sXI + c.t * XJ, zj = tXI + c.s * XJ;
            const double fval = pt(k, zi, zj);
            double pa, f1, f2;
            if (r <= H) {
                pa = p - p * tab[tab_at(TL_A, k)];
                const double q = div_rcp(tab[tab_at(TL_M, k)], c.sqrtpr, c.rsqrtpr);
                f1 = tab[tab_at(TL_A1, k)] + q;
                f2 = tab[tab_at(TL_A1, k)] - q;
                if (r < H) { pA[r] = pa; F1[r] = f1; F2[r] = f2; }
            } else {
                pa = pA[KK - 1 - r];
                f1 = F1[KK - 1 - r];
                f2 = F2[KK - 1 - r];
            }
            S.dp = S.dp + fval * (pa + tab[tab_at(TL_X2, k)]);
            S.du1 = S.du1 + fval * (zi - p * zj);
            S.du2 = S.du2 + fval * (zj - p * zi);
            S.do1 = S.do1 + fval * f1;
            S.do2 = S.do2 + fval * f2;
            S.Ei = S.Ei + fval;
        }
    }
}

// The node gradient's loop at K = 9 with the rows unrolled GQ_LIT_NODE_UNROLL
// times (1: the runtime-K loop): the next point's tap gathers can then issue
// before this point's taps are summed.  The same operations in the same order.
// Measured 2 / 3: 297.8 / 298.2 against 268.1 us (register pressure at the
// 3-wave bound; profiles/r06_lit_minmax_addr_ab.txt): not used.
#ifndef GQ_LIT_NODE_UNROLL
#define GQ_LIT_NODE_UNROLL 1
#endif
template <int KK, typename TP, typename PT>
GQ_HD void lit_points_fixed(TP tab, const LitCoef &c, double p, LitAcc &S, PT pt)
{
    for (int cc = 0, k0 = 0; cc < KK; ++cc, k0 += KK) {
        const double XI = tab[tab_at(TL_XI, k0)];
        const double sXI = c.s * XI, tXI = c.t * XI;
#ifdef __HIPCC__
#pragma unroll GQ_LIT_NODE_UNROLL
#endif
        for (int r = 0; r < KK; ++r) {
            const int k = k0 + r;
            const double XJ = tab[tab_at(TL_XJ, k)];
            const double zi = sXI + c.t * XJ, zj = tXI + c.s * XJ;
            S.add(tab, k, pt(k, zi, zj), zi, zj, p, c.sqrtpr, c.rsqrtpr, true);
        }
    }
}

template <typename TP, typename PT>
GQ_HD void lit_points_dyn(TP tab, int K2, const LitCoef &c, double p, LitAcc &S, PT pt, bool live)
{
#if GQ_LIT_CSE
    const int K = lit_k(K2);
    for (int cc = 0, k = 0; cc < K; ++cc) {
        const double XI = tab[tab_at(TL_XI, k)];
        const double sXI = c.s * XI, tXI = c.t * XI;
        for (int r = 0; r < K; ++r, ++k) {
            const double XJ = tab[tab_at(TL_XJ, k)];
            const double zi = sXI + c.t * XJ, zj = tXI + c.s * XJ;
            S.add(tab, k, pt(k, zi, zj), zi, zj, p, c.sqrtpr, c.rsqrtpr, live);
        }
    }
#else
    for (int k = 0; k < K2; ++k) {
        const double XI = tab[tab_at(TL_XI, k)], XJ = tab[tab_at(TL_XJ, k)];
        const double zi = c.s * XI + c.t * XJ, zj = c.t * XI + c.s * XJ;
        S.add(tab, k, pt(k, zi, zj), zi, zj, p, c.sqrtpr, c.rsqrtpr, live);
    }
#endif
}

template <typename TP, typename PT>
GQ_HD void lit_loop(TP tab, int K2, const LitCoef &c, double p, bool live, LitAcc &S, PT pt)
{
#if GQ_LIT_HOIST
    if (live) lit_points<true>(tab, K2, c, p, S, pt);
    else lit_points<false>(tab, K2, c, p, S, pt);
#else
    // `live` tested at every point (LitAcc::add)
    lit_points_dyn(tab, K2, c, p, S, pt, live);
#endif
}

// node_grad_spectral with node_pot, (m, n) 0-based pixel of the frame
template <typename TP, typename VP, typename IP>
GQ_HD Grad<double> lit_node_grad(TP tab, int K2, VP VV, int M2, IP I1, int Mo, int No, double eps, double lamd,
                                 bool guard, double T, double a, double u1, double u2, double o1, double o2, double p,
                                 int m, int n)
{
    const LitCoef c = lit_coef(p);
    const double so1 = GQ_M_SQRT2 * o1, so2 = GQ_M_SQRT2 * o2;
    const double I = I1[m + (int64_t)Mo * n];
    const bool live = !guard || a != 0;
    LitAcc S;
    auto pt = [&](int k, double zi, double zj) {
        const double x1 = so1 * zi + u1, x2 = so2 * zj + u2;
        const double d = I - lit_interp(VV, M2, Mo, No, (double)(n + 1) + x1, (double)(m + 1) + x2);
        return tab[tab_at(TL_W, k)] * (-lamd * GQ_SQRT(eps + d * d));
    };
#if GQ_LIT_MIRROR && GQ_LIT_MIRROR_NODE
    if (K2 == 81 && live) lit_points_mirror<9>(tab, c, p, S, pt);
    else
#elif GQ_LIT_NODE_UNROLL > 1
    if (K2 == 81 && live) lit_points_fixed<9>(tab, c, p, S, pt);
    else
#endif
        lit_loop(tab, K2, c, p, live, S, pt);
    return lit_epi(S, c, a, o1, o2, p, T, true);
}

// edge_grad_spectral with edge_pot
template <typename TP>
GQ_HD Grad<double> lit_edge_grad(TP tab, int K2, double eps, double lams, bool guard, double T, double a, double u1,
                                 double u2, double o1, double o2, double p)
{
    const LitCoef c = lit_coef(p);
    const double so1 = GQ_M_SQRT2 * o1, so2 = GQ_M_SQRT2 * o2;
    const bool live = !guard || a != 0;
    LitAcc S;
    auto pt = [&](int k, double zi, double zj) {
        const double d = (so1 * zi + u1) - (so2 * zj + u2);
        return tab[tab_at(TL_W, k)] * (-lams * GQ_SQRT(eps + d * d));
    };
#if GQ_LIT_MIRROR
    if (K2 == 81 && live) lit_points_mirror<9>(tab, c, p, S, pt);
    else
#endif
        lit_loop(tab, K2, c, p, live, S, pt);
    return lit_epi(S, c, a, o1, o2, p, T, false);
}

}  // namespace gq
