// cwbl_device.h — device helpers shared by the HIP kernels of the LETKF core:
// reference-exact fp32 weight functions, fp64 reciprocal helpers, cross-lane reductions,
// and the column-assembly stage of the per-point solve (Yb Yb^T and Yb d in fp64).
#pragma once

#include "cwbl_internal.h"

#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

namespace cwbl {

// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>), in order: compile-time
// blocking of loops whose bodies pick registers or LDS offsets by the index
template <int... Is, class F>
__device__ __forceinline__ void sfor_impl(std::integer_sequence<int, Is...>, F &&f) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F &&f) {
  sfor_impl(std::make_integer_sequence<int, N>{}, f);
}

// ---------------------------------------------------------------------------------------
// fp32 helpers that must round exactly like the reference build
// ---------------------------------------------------------------------------------------
static __constant__ unsigned long long kExpT[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

// exp(real(4)) as the reference build evaluates it: glibc 2.35 expf, FMA variant
// (table-driven, computed in double; the reference's flang `exp` calls libm expf).
// Attribution: the table kExpT and the polynomial constants below are those of glibc's
// sysdeps/ieee754/flt-32/e_expf.c / e_exp2f_data.c (Szabolcs Nagy, ARM Ltd., 2017; GNU
// LGPL 2.1+), reproduced so that the weight 1/(err * exp(r2/4)) rounds exactly as the
// reference's does (module_letkf_core.f90:444; checked on all floats in [0, 8),
// oracle/tools/expf_check.c).
__device__ __forceinline__ float expf_ref(float x, const unsigned long long *tab = kExpT) {
  const unsigned ux = __float_as_uint(x);
  const unsigned abstop = (ux >> 20) & 0x7ffu;
  if (abstop >= 0x42bu) {  // |x| >= 88: not reached on this path (0.25*r2 <= 3.34)
    if (ux == 0xff800000u) return 0.0f;
    return expf(x);
  }
  const double shift = __longlong_as_double(0x4338000000000000ll);
  const double invln2n = __longlong_as_double(0x40471547652b82fell);
  const double c0 = __longlong_as_double(0x3ebc6af84b912394ll);
  const double c1 = __longlong_as_double(0x3f2ebfce50fac4f3ll);
  const double c2 = __longlong_as_double(0x3f962e42ff0c52d6ll);
  const double xd = (double)x;
  double kd = fma(invln2n, xd, shift);
  const unsigned long long ki = (unsigned long long)__double_as_longlong(kd);
  kd = kd - shift;
  const double r = fma(invln2n, xd, -kd);
  unsigned long long t = tab[ki & 31ull];
  t += ki << 47;
  const double s = __longlong_as_double((long long)t);
  const double z = fma(r, c0, c1);
  const double r2 = r * r;
  double y = fma(r, c2, 1.0);
  y = fma(z, r2, y);
  y = y * s;
  return (float)y;
}

// Gaspari_Cohn_1999, module_localization.f90:333-364 (fp32, unfused)
__device__ __forceinline__ float gaspari_cohn(float x) {
  const float a = 1.82574189f;  // sqrt(10./3.) in fp32 (== sqrtf(10.0f/3.0f))
  const float a1 = -0.25f, a2 = 0.5f, a3 = 0.625f, a4 = -5.0f / 3.0f, a5 = 1.0f;
  const float b1 = 1.0f / 12.0f, b2 = -0.5f, b3 = 0.625f, b4 = 5.0f / 3.0f, b5 = -5.0f,
              b6 = 4.0f, b7 = -2.0f / 3.0f;
  const float z = x / a;
  if (z <= 1.0f) return z * z * (z * (z * (a1 * z + a2) + a3) + a4) + a5;
  if (z <= 2.0f) return z * (z * (z * (z * (b1 * z + b2) + b3) + b4) + b5) + b6 + b7 / z;
  return 0.0f;
}

// localisation weight on the error, module_letkf_core.f90:443-450 / 516-523
__device__ __forceinline__ float error_inv(int wf, float err, float r2,
                                           const unsigned long long *tab = kExpT) {
  if (wf != 1) return 1.0f / (err * expf_ref(0.25f * r2, tab));
  return sqrtf(gaspari_cohn(sqrtf(r2))) / err;
}


// ---------------------------------------------------------------------------------------
// fp64 helpers
// ---------------------------------------------------------------------------------------
// fp64 reciprocal / reciprocal square root: hardware estimate + two Newton steps (~1 ulp).
// The rotation only needs c^2 + s^2 = 1 to working precision, not IEEE-rounded c and s.
__device__ __forceinline__ double rcp64(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}
__device__ __forceinline__ double rsq64(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  double t = fma(-h * y, y, 0.5);
  y = fma(y, t, y);
  t = fma(-h * y, y, 0.5);
  return fma(y, t, y);
}

__device__ __forceinline__ int xcd_remap(int b, int n) {
  const int x = b & 7, l = b >> 3, q = n >> 3, r = n & 7;
  return x * q + (x < r ? x : r) + l;
}
// the same chunks, each walked from its end
__device__ __forceinline__ int xcd_remap_rev(int b, int n) {
  const int x = b & 7, l = b >> 3, q = n >> 3, r = n & 7;
  return x * q + (x < r ? x : r) + (q + (x < r ? 1 : 0) - 1 - l);
}

__device__ __forceinline__ double wave_sum_f64(double v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// DPP lane exchange of a double (two 32-bit moves).  Callers keep all 64 lanes active.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double readlane_f64(double x, int l) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// ---- 16-lane row broadcasts (gfx950's 64-bit DPP is row_newbcast only) ------------------
// value of lane L of this lane's 16-lane row (one v_mov_b64 DPP; bound_ctrl: every source
// lane is active)
template <int L>
__device__ __forceinline__ double rbcast(double x) {
  return __longlong_as_double(
      __builtin_amdgcn_update_dpp(0ll, __double_as_longlong(x), 0x150 + L, 0xf, 0xf, true));
}
template <int L>
__device__ __forceinline__ float rbcast(float x) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x150 + L, 0xf, 0xf, true));
}
// acc + x_L y and acc - x_L y, x_L = lane L of this lane's 16-lane row: one v_fmac_f64_dpp
// row_newbcast instead of a v_mov_b64_dpp broadcast and an FMA.  The compiler does not form
// it itself (its DPP combine sees the three-address v_fma_f64).  A DPP source must not be
// written by the VALU in the two instructions before: callers write their sources once and
// pin them behind an s_nop 1 (dpp_pin) before the first use; the compiler's hazard check
// covers the inline asm's other operands.
template <int L>
__device__ __forceinline__ double fmac_row(double acc, double x, double y) {
  asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : "+v"(acc) : "v"(x), "v"(y), "i"(L));
  return acc;
}
template <int L>
__device__ __forceinline__ double fnmac_row(double acc, double x, double y) {
  asm("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : "+v"(acc) : "v"(x), "v"(y), "i"(L));
  return acc;
}
__device__ __forceinline__ void dpp_pin(double &x) { asm volatile("s_nop 1" : "+v"(x)); }
// the same as volatile statements: kept in program order relative to each other and to the
// volatile s_nop that opens a pass (dpp_fence), so no VALU write of a DPP source lands within
// two instructions of its read
template <int L>
__device__ __forceinline__ double fmac_row_v(double acc, double x, double y) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
               : "+v"(acc) : "v"(x), "v"(y), "i"(L));
  return acc;
}
template <int L>
__device__ __forceinline__ double fnmac_row_v(double acc, double x, double y) {
  asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
               : "+v"(acc) : "v"(x), "v"(y), "i"(L));
  return acc;
}
__device__ __forceinline__ void dpp_fence() { asm volatile("s_nop 1" ::: "memory"); }
// value of lane l ^ 8 of the row (row_ror:8)
__device__ __forceinline__ double ror8(double x) { return dpp_f64<0x128>(x); }
// sum over each 8-lane half of a 16-lane row (quad sums, then the half mirror)
__device__ __forceinline__ double rsum8(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  return v;
}

// ---- per-point records through a buffer resource ----------------------------------------
// A lane whose byte offset is kRecSkip (past any record) loads 0 and stores nothing, with no
// memory access: triangular parts of a record are masked without branches (a branch around
// a load leaves the wait for it on the skipping path) and without moving their zero bytes.
constexpr unsigned kRecSkip = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rec_rsrc(const double *base, int words) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(base), 0, words * 8, 0x00020000);
}
// word w of the record, or kRecSkip
__device__ __forceinline__ unsigned rec_off(bool live, int w) {
  return live ? 8u * (unsigned)w : kRecSkip;
}
__device__ __forceinline__ double rec_ld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
  return __longlong_as_double(((long long)v[1] << 32) | (unsigned)v[0]);
}
__device__ __forceinline__ void rec_st(__amdgpu_buffer_rsrc_t r, unsigned off, double x) {
  const long long b = __double_as_longlong(x);
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 v = {(unsigned)b, (unsigned)(b >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)off, 0, 0);
}

// v through a register the compiler cannot see through, after `dep` is known.  The per-row
// LDS offsets of a quadrature walk whose direction differs per lane (base + dir * t) are
// loop-invariant: without this the compiler hoists all of them out of the pass loop and holds
// one VGPR per row; formed from an opaque base they are computed where they are used.
__device__ __forceinline__ unsigned opaque_after(unsigned v, double dep) {
  asm volatile("" : "+v"(v) : "v"(dep));
  return v;
}
// the double at byte offset `off` of a shared-memory object
__device__ __forceinline__ double lds_at(const void *base, unsigned off) {
  return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(base) + off);
}

// v through a register the compiler cannot see through: values formed from it are formed
// where they are used instead of being hoisted out of the loop around them (and held)
__device__ __forceinline__ int opaque_int(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Sum over each 16-lane row; every lane of a row gets the same (bitwise) row sum.
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  v += dpp_f64<0x140>(v);  // row_mirror
  return v;
}

// x[lane] + x[lane ^ 16] (PERM = 16) or x[lane] + x[lane ^ 32] (PERM = 32) with gfx950's
// v_permlane{16,32}_swap; both lanes of a pair add in the same order (bitwise equal sums).
template <int PERM>
__device__ __forceinline__ double swap_add_f64(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = (int)b, hi = (int)(b >> 32);
  auto rl = PERM == 16 ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false)
                       : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  auto rh = PERM == 16 ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false)
                       : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const double a = __longlong_as_double(((long long)rh[0] << 32) | (unsigned)rl[0]);
  const double c = __longlong_as_double(((long long)rh[1] << 32) | (unsigned)rl[1]);
  return a + c;
}

// Sum over the 64 lanes, the same value in every lane.
__device__ __forceinline__ double wave_sum_dpp(double v) {
  return swap_add_f64<32>(swap_add_f64<16>(row16_sum(v)));
}

// Four wave sums at once: two transposing stages (v_permlane32_swap, v_permlane16_swap)
// leave row r of the wave holding partial sums of value r, a row reduction finishes them,
// and lanes 0/16/32/48 hand the results out as wave-uniform values.  29 instructions for
// four sums instead of 4 x 22.
__device__ __forceinline__ void wave_sum4_dpp(double &a, double &b, double &c, double &d) {
  auto lo = [](double x) { return (int)__double_as_longlong(x); };
  auto hi = [](double x) { return (int)(__double_as_longlong(x) >> 32); };
  auto mk = [](int l, int h) { return __longlong_as_double(((long long)h << 32) | (unsigned)l); };
  // lanes 0-31: a[i] + a[i+32], lanes 32-63: c[i-32] + c[i]; same for (b, d)
  auto s1l = __builtin_amdgcn_permlane32_swap(lo(a), lo(c), false, false);
  auto s1h = __builtin_amdgcn_permlane32_swap(hi(a), hi(c), false, false);
  auto s2l = __builtin_amdgcn_permlane32_swap(lo(b), lo(d), false, false);
  auto s2h = __builtin_amdgcn_permlane32_swap(hi(b), hi(d), false, false);
  const double r1 = mk(s1l[0], s1h[0]) + mk(s1l[1], s1h[1]);
  const double r2 = mk(s2l[0], s2h[0]) + mk(s2l[1], s2h[1]);
  // even rows: r1[i] + r1[i+16], odd rows: r2[i-16] + r2[i] -> row 0 a, 1 b, 2 c, 3 d
  auto tl = __builtin_amdgcn_permlane16_swap(lo(r1), lo(r2), false, false);
  auto th = __builtin_amdgcn_permlane16_swap(hi(r1), hi(r2), false, false);
  const double r = row16_sum(mk(tl[0], th[0]) + mk(tl[1], th[1]));
  a = readlane_f64(r, 0);
  b = readlane_f64(r, 16);
  c = readlane_f64(r, 32);
  d = readlane_f64(r, 48);
}

// Sum over each half wave (lanes 0-31, 32-63); every lane gets its half's sum.
__device__ __forceinline__ double half_sum_dpp(double v) {
  return swap_add_f64<16>(row16_sum(v));
}

// Generic pointers held in structs (TreeDesc, SlabDev) are global memory; saying so lets the
// compiler emit global_load (vector memory only) instead of flat loads, which also wait on
// the LDS counter.
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T *gptr(const T *p) {
  return (const __attribute__((address_space(1))) T *)p;
}
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 gload4(const float *p) {  // 16-B global load
  return *gptr(reinterpret_cast<const f32x4 *>(p));
}
// base[i] with a 32-bit byte offset (SGPR base + VGPR offset addressing); tables < 4 GiB
template <class T>
__device__ __forceinline__ T gld(const T *base, unsigned i) {
  const char *b = reinterpret_cast<const char *>(base) + (unsigned)(i * (unsigned)sizeof(T));
  return *gptr(reinterpret_cast<const T *>(b));
}
// *(T *)((char *)base + byteoff) = v, a global store at SGPR base + 32-bit offset
template <class T>
__device__ __forceinline__ void gst(T *base, unsigned byteoff, T v) {
  char *b = reinterpret_cast<char *>(base) + byteoff;
  *(__attribute__((address_space(1))) T *)reinterpret_cast<T *>(b) = v;
}
__device__ __forceinline__ f32x4 gld4(const float *base, unsigned i) {  // 16 B at base + 4i
  const char *b = reinterpret_cast<const char *>(base) + (unsigned)(i * 4u);
  return *gptr(reinterpret_cast<const f32x4 *>(b));
}

// Grid point g of a slab (the enumeration g = i + ix_lim*(j + iy_lim*kz) of the reference's
// point loop, module_letkf_core.f90:209-213): projected x, y and altitude.
// (g < 2^32: cwbl_analyze_var rejects larger slabs, so the divisions are 32-bit)
__device__ __forceinline__ void slab_point(const SlabDev &s, long long g, float &x, float &y,
                                           float &z) {
  const unsigned gg = (unsigned)g, ix = (unsigned)s.ix_lim, iy = (unsigned)s.iy_lim;
  const unsigned r = gg / ix, i = gg - r * ix, kz = r / iy, j = r - kz * iy;
  x = gptr(s.x)[i + (long long)s.nx * j];
  y = gptr(s.y)[i + (long long)s.nx * j];
  z = gptr(s.alt)[i + (long long)s.alt_nx * (j + (long long)s.alt_ny * kz)];
}

// Squared normalised distance of a tree point (rearranged coordinates d) from the normalised
// query (q0, q1, q2), evaluated exactly as the search does (process_terminal_node_fixedball,
// module_kdtree2.f90:1654-1707), so the solve reproduces the search's r2 bit for bit.
__device__ __forceinline__ float slot_r2(const f32x4 d, int dim, float q0, float q1,
                                         float q2) {
  const float dx = d.x - q0, dy = d.y - q1;
  float sd = dx * dx;
  sd = sd + dy * dy;
  if (dim == 3) {
    const float dz = d.z - q2;
    sd = sd + dz * dz;
  }
  return sd;
}

// ---------------------------------------------------------------------------------------
// Column assembly of one grid point (one wavefront): the point-dependent half of
// letkf_yoyb (localisation weight on the error, module_letkf_core.f90:443-452) fused with
// the Yb Yb^T (dsyrk) and Yb d products of letkf_solve (:598-700), in fp64.
// Lane L owns the 4x4 blocks L, L+64, ... of the lower block triangle (bi >= bj).
// ---------------------------------------------------------------------------------------
// Staged columns: E = float (converted by the consumer) or double (converted once here;
// products of the fp32 values stay exact in fp64 either way).
// PITCH > KP (the matrix-core assembly): a staged column also holds yo in row KP and zeros
// in rows KP+1 .. PITCH-1, so the MFMA operand rows [Yb; yo; 0] read without selects.
// SWZ (matrix-core pitches with PITCH % 32 == 16): column s starts 2 (s >> 1) words after
// s * PITCH.  The pair staging's 8-byte stores (16 lanes = 16 columns at one row offset) then
// hit 16 distinct bank pairs instead of 2 (8-way conflicts: ~2.6 k extra LDS cycles per
// point), and the MFMA operand reads, whose two 32-lane groups read columns 4g, 4g + 1 and
// 4g + 2, 4g + 3 (same shift, bases 16 banks apart), stay conflict-free.  Columns keep all
// PITCH rows (the shifts grow with s), so the chunk takes CHUNK more words.
//
// XSW (the 256-thread kernels' chunks, PITCH = 128): row r of an odd column is stored at
// r ^ 16.  Their MFMA operand reads (two 32-lane groups, columns 4g + kk, rows 16 x + m) then
// put the odd column 16 banks away from the even one instead of on the same banks (2-way),
// and with the staging stores' rotated order (stage_columns_pipe) the stores of 16 lanes
// (16 columns) spread over the banks instead of all hitting one (16-way); no extra LDS.
template <int KP, int CHUNK, class E = float, int PITCH = KP, bool SWZ = false, bool XSW = false>
struct ColumnChunk {
  E yb[CHUNK][PITCH];
  E yb_shift[SWZ ? CHUNK : 1];  // room for the shifted columns (SWZ)
  E yo[CHUNK];
  unsigned long long expt[32];  // expf table (kExpT) in LDS: per-lane lookups stay on chip
  // col(s + 4) = col(s) + GSTRIDE: the MFMA group loops step from col(kk) by it, so that the
  // compiler sees one base and immediate offsets
  static constexpr int GSTRIDE = 4 * PITCH + (SWZ ? 4 : 0);
  __device__ __forceinline__ E *col(int s) {
    return reinterpret_cast<E *>(this) + s * PITCH + (SWZ ? 2 * (s >> 1) : 0);
  }
  __device__ __forceinline__ const E *col(int s) const {
    return reinterpret_cast<const E *>(this) + s * PITCH + (SWZ ? 2 * (s >> 1) : 0);
  }
  static __device__ __forceinline__ int xr(int s) { return XSW ? 16 * (s & 1) : 0; }
  __device__ __forceinline__ E &at(int s, int row) { return col(s)[row ^ xr(s)]; }
  __device__ __forceinline__ const E &at(int s, int row) const { return col(s)[row ^ xr(s)]; }
};

template <int KP, int NT = 64>
struct AsmLayout {
  static constexpr int NB = KP / 4;                 // 4x4 blocks per dimension
  static constexpr int NBLK = NB * (NB + 1) / 2;    // lower-triangle blocks
  static constexpr int NBL = (NBLK + NT - 1) / NT;  // blocks per thread (NT threads per point)
};

// Stages the point's columns CHUNK at a time into `ch` (yb = bg * error_inv,
// yo = omm * error_inv, in the reference's fp32 order; rejected columns as zeros) and calls
// accumulate(nsl) on each staged chunk.  NT threads per point (`lane` = thread index).
// Returns the number of accepted columns (p); with NT > 64 the count is valid in wave 0.
template <int KP, int CHUNK, bool ASSEMBLED, int NT = 64, class E = float, int PITCH = KP,
          bool SWZ = false, bool XSW = false, class Acc>
__device__ __forceinline__ int stage_columns(
    ColumnChunk<KP, CHUNK, E, PITCH, SWZ, XSW> &ch, const TreeDesc *__restrict__ trees, const SolveConsts &c,
    int gi, int lane, const int *__restrict__ nbr_cnt, const int *__restrict__ nbr_idx,
    const float3 pt, const long long *__restrict__ col_off,
    const float *__restrict__ yo_in, const float *__restrict__ yb_in, Acc &&accumulate) {
  const int k = c.k;
  int ptot = 0;
  if constexpr (!ASSEMBLED) {
    if (lane < 32) ch.expt[lane] = kExpT[lane];
    if constexpr (PITCH > KP + 1) {  // rows KP+1 .. PITCH-1 of every column stay zero
      constexpr int NZ = PITCH - KP - 1;
      for (int e = lane; e < CHUNK * NZ; e += NT) ch.at(e / NZ, KP + 1 + e % NZ) = (E)0.0f;
    }
    // other waves read the table before the chunk loop's first barrier (error_inv below);
    // LDS is not cleared between workgroups, so without this they can read a previous
    // workgroup's bytes (one wave: the lanes' LDS ops are ordered, no barrier needed)
    if constexpr (NT > 64) __syncthreads();
    for (int t = 0; t < c.ntrees; ++t) {
      const TreeDesc T = trees[t];  // by value: the fields live in SGPRs for the whole loop
      // get_lz normalisation of the point (module_localization.f90:243-253), as the search
      const float q0 = pt.x * T.hclr_inv, q1 = pt.y * T.hclr_inv;
      const float q2 = T.query3d ? pt.z * T.vclr_inv : 0.0f;
      const int cnt = gptr(nbr_cnt)[(long long)gi * c.ntrees + t];
      const int nvar = T.nvar;
      const int npairs = cnt * nvar;
      const long long lbase = list_index(gi, c.list_cap, T.list_off);
      // Candidate columns stay in the search's order; a rejected one is staged as a zero
      // column (its bg row is zero and its weight 0), which adds exact zeros to every sum.
      // So every gather of a chunk depends only on the neighbour slots: one round trip to
      // memory per chunk, with the next chunk's slots prefetched behind it.  Threads s,
      // s + CHUNK, s + 2 CHUNK, ... stage column s of the chunk, a part of its bg row each.
      static_assert(NT % CHUNK == 0 && CHUNK <= 64, "threads per staged column");
      constexpr int LPC = NT / CHUNK;                    // threads per staged column
      constexpr int VH = KP / (2 * LPC);                 // float2 of the bg row per thread
      static_assert(KP % (2 * LPC) == 0, "bg row split");
      const int sl = lane % CHUNK, half = lane / CHUNK;
      const int *__restrict__ lst = nbr_idx + lbase;
      // q / nvar for the (obs, variable) pair index q < 2^22: a float estimate and one
      // correction each way (nvar is wave-uniform; 1 for radar)
      const float rnv = 1.0f / (float)nvar;
      auto divn = [&](int q) {
        if (nvar == 1) return q;  // radar (wave-uniform): no division
        int j = (int)((float)q * rnv);
        j -= j * nvar > q ? 1 : 0;
        j += (j + 1) * nvar <= q ? 1 : 0;
        return j;
      };
      int slot_next = 0;
      if (sl < min(CHUNK, npairs)) slot_next = gld(lst, list_slot(divn(sl)));
      for (int base = 0; base < npairs; base += CHUNK) {
        const int nsl = min(CHUNK, npairs - base);
        const bool live = sl < nsl;
        const int q = base + sl;
        const int jn = divn(q), v = q - jn * nvar;
        const int slot = slot_next;
        const int col = slot * nvar + v;
        // the next chunk's slot first: it depends on nothing gathered below.  The load is
        // unconditional (a lane past the list, or every lane on the last chunk, reads the
        // slot of pair npairs - 1: a valid table index whose column w = 0 zeroes): behind a
        // branch, the skipping path left the wait for the gathers' operands at vmcnt(0), so
        // the gathers waited a whole round trip for this prefetch.
        const int nb = base + CHUNK;
        slot_next = gld(lst, list_slot(divn(min(nb + sl, npairs - 1))));
        // Gathers without a branch: a lane past nsl keeps the slot of an earlier chunk (or
        // 0), a valid table index, and its column is zeroed by w = 0 below.  The bg row part
        // goes first and as 16-B loads (b0 is a multiple of 4 floats: KP % 8 == 0), then
        // the scalars; all addresses are formed before the first load.
        float2 g[VH];
        const unsigned b0 = (unsigned)(col * KP + 2 * VH * half);
        if constexpr (VH % 2 == 0) {
#pragma unroll
          for (int i = 0; i < VH / 2; ++i) {
            const f32x4 t = gld4(T.col_bg, b0 + 4u * i);
            g[2 * i] = make_float2(t.x, t.y);
            g[2 * i + 1] = make_float2(t.z, t.w);
          }
        } else {
          typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
          for (int i = 0; i < VH; ++i) {
            const char *bp = reinterpret_cast<const char *>(T.col_bg) + (unsigned)((b0 + 2u * i) * 4u);
            const f32x2 t = *gptr(reinterpret_cast<const f32x2 *>(bp));
            g[i] = make_float2(t.x, t.y);
          }
        }
        const uint8_t okb = gld(T.col_ok, (unsigned)col);
        const float err = gld(T.col_err, (unsigned)col);
        const float omm = gld(T.col_omm, (unsigned)col);
        const f32x4 rd = gld4(reinterpret_cast<const float *>(T.rdata), 4u * (unsigned)slot);
        const bool ok = live && okb != 0;
        // computed for every lane and selected (a branch here would sink the rd/err/omm
        // loads behind the ok-flag load: two round trips per chunk instead of one)
        const float wv =
            error_inv(c.weight_function, err, slot_r2(rd, T.tree_dim, q0, q1, q2), ch.expt);
        const float w = ok ? wv : 0.0f;
        const float yo = ok ? omm * wv : 0.0f;  // omm * error_inv (:451)
        ptot += __popcll(__ballot(ok && half == 0));  // counted by wave 0
        if (half == 0) {
          ch.yo[sl] = (E)yo;
          if constexpr (PITCH > KP) ch.at(sl, KP) = (E)yo;
        }
#pragma unroll
        for (int i = 0; i < VH; ++i) {
          // bg * error_inv (:452); w = 0 zeroes a rejected column and a lane past nsl (its
          // bg is a finite table entry of an earlier slot)
          const float y0 = g[i].x * w, y1 = g[i].y * w;
          E *dst = &ch.at(sl, 2 * VH * half + 2 * i);  // (an aligned pair under XSW too)
          if constexpr (sizeof(E) == 8) {
            *reinterpret_cast<double2 *>(dst) = make_double2((double)y0, (double)y1);
          } else {
            *reinterpret_cast<float2 *>(dst) = make_float2(y0, y1);
          }
        }
        __syncthreads();
        accumulate(nsl);
        __syncthreads();
      }
    }
  } else {
    const long long c0 = col_off[gi], c1 = col_off[gi + 1];
    const int ncol = (int)(c1 - c0);
    for (int base = 0; base < ncol; base += CHUNK) {
      const int nsl = min(CHUNK, ncol - base);
      // the whole chunk is written (zeros past nsl), as on the analysis path
      if (lane < CHUNK) ch.yo[lane] = lane < nsl ? (E)yo_in[c0 + base + lane] : (E)0.0f;
      for (int e = lane; e < CHUNK * PITCH; e += NT) {
        const int s = e / PITCH, m = e - s * PITCH;
        E v = (E)0.0f;
        if (s < nsl) {
          if (m < k) v = (E)yb_in[(c0 + base + s) * k + m];
          else if (m == KP) v = (E)yo_in[c0 + base + s];  // PITCH > KP only
        }
        ch.at(s, m) = v;
      }
      __syncthreads();
      accumulate(nsl);
      ptot += nsl;
      __syncthreads();
    }
  }
  return ptot;
}

// The value of lane i ^ 32 (the other half wave), by one v_permlane32_swap.
__device__ __forceinline__ int other_half(int x, int half) {
  const auto s = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return half ? s[0] : s[1];  // s[0]: lanes 32-63 get x[i-32]; s[1]: lanes 0-31 get x[i+32]
}
__device__ __forceinline__ float other_half(float x, int half) {
  return __int_as_float(other_half(__float_as_int(x), half));
}

// stage_columns for one wavefront, CHUNK = 32, analysis path, two chunks per round: the
// weight of a column is computed once, not by both lanes that stage its bg row.  Lane
// (half, sl) owns column sl of chunk c + half (its slot, QC flag, error, omm, coordinates,
// weight) and stages half `half` of the bg row of column sl of chunk c, then of chunk c + 1;
// the weight of the column it stages but does not own comes from lane sl + 32 (half 0) or
// sl (half 1) by one swap.  Same columns, order and arithmetic as stage_columns.
// `side` may stage part of each column a second time, elsewhere (the record kernel's fp64
// rows): side.stage(half, sl, g, w) sees every lane's gathered bg quads and weight right
// after they are staged, side.yo(sl, yo) every staged yo.
struct NoSide {
  static constexpr bool kPad = true;  // zero the chunk's padding rows KP + 1 .. PITCH - 1
  template <class G>
  __device__ __forceinline__ void stage(int, int, const G &, float) {}
  __device__ __forceinline__ void yo(int, float) {}
};
template <int KP, int CHUNK, int PITCH, bool SWZ, bool XSW = false, class Acc,
          class Side = NoSide>
__device__ __forceinline__ int stage_columns_pair(
    ColumnChunk<KP, CHUNK, float, PITCH, SWZ, XSW> &ch, const TreeDesc *__restrict__ trees,
    const SolveConsts &c, int gi, int lane, const int *__restrict__ nbr_cnt,
    const int *__restrict__ nbr_idx, const float3 pt, Acc &&accumulate, Side &&side = Side{}) {
  static_assert(CHUNK == 32, "two lanes per staged column");
  constexpr int VH = KP / 4;  // float2 of the bg row per lane
  static_assert(KP % 8 == 0, "bg row split into 16-B loads");
  int ptot = 0;
  if (lane < 32) ch.expt[lane] = kExpT[lane];
  if constexpr (PITCH > KP + 1 && std::decay_t<Side>::kPad) {
    constexpr int NZ = PITCH - KP - 1;
    for (int e = lane; e < CHUNK * NZ; e += 64) ch.at(e / NZ, KP + 1 + e % NZ) = 0.0f;
  }
  const int sl = lane % CHUNK, half = lane / CHUNK;
  // XSW (pitches 32, 64): the lane gathers and stores its VH / 2 float4 starting at float4
  // (sl >> 1) mod VH / 2, so a 16-lane store group writes several row offsets, with the odd
  // columns' r ^ 16 on top (ColumnChunk), instead of one
  constexpr int NQ = VH / 2;
  const int rot = XSW ? (sl >> 1) % NQ : 0;
  auto quad = [&](int i) { return XSW ? (i + rot >= NQ ? i + rot - NQ : i + rot) : i; };
  for (int t = 0; t < c.ntrees; ++t) {
    const TreeDesc T = trees[t];
    const float q0 = pt.x * T.hclr_inv, q1 = pt.y * T.hclr_inv;  // get_lz (:243-253)
    const float q2 = T.query3d ? pt.z * T.vclr_inv : 0.0f;
    const int cnt = gptr(nbr_cnt)[(long long)gi * c.ntrees + t];
    const int nvar = T.nvar;
    const int npairs = cnt * nvar;
    if (npairs == 0) continue;
    const int *__restrict__ lst = nbr_idx + list_index(gi, c.list_cap, T.list_off);
    const float rnv = 1.0f / (float)nvar;
    auto divn = [&](int q) {
      if (nvar == 1) return q;
      int j = (int)((float)q * rnv);
      j -= j * nvar > q ? 1 : 0;
      j += (j + 1) * nvar <= q ? 1 : 0;
      return j;
    };
    // a lane past the list reads the slot of pair npairs - 1 (a valid table index; the
    // column's weight is 0)
    auto slot_at = [&](int q) { return gld(lst, list_slot(divn(min(q, npairs - 1)))); };
    auto var_of = [&](int q) { return q - divn(q) * nvar; };
    auto gather_bg = [&](int col, f32x4 (&g)[VH / 2]) {
      const unsigned b0 = (unsigned)(col * KP + 2 * VH * half);
      if (CWBL_DBG_STOP(c) == 13) {  // timing ablation: the assembly without the gathers
#pragma unroll
        for (int i = 0; i < VH / 2; ++i) g[i] = f32x4{1.0f, 1.0f, 1.0f, 1.0f};
        return;
      }
#pragma unroll
      for (int i = 0; i < VH / 2; ++i) g[i] = gld4(T.col_bg, b0 + 4u * (unsigned)quad(i));
    };
    auto put = [&](const f32x4 (&g)[VH / 2], float w) {  // bg * error_inv (:452)
#pragma unroll
      for (int i = 0; i < VH / 2; ++i) {
        const int r = 2 * VH * half + 4 * quad(i);
        *reinterpret_cast<float2 *>(&ch.at(sl, r)) = make_float2(g[i].x * w, g[i].y * w);
        *reinterpret_cast<float2 *>(&ch.at(sl, r + 2)) = make_float2(g[i].z * w, g[i].w * w);
      }
    };
    int slot_next = slot_at(half * CHUNK + sl);
    for (int base = 0; base < npairs; base += 2 * CHUNK) {
      const int qo = base + half * CHUNK + sl;  // the owned column's pair index
      const int slot = slot_next;
      slot_next = slot_at(qo + 2 * CHUNK);      // the next round's, behind nothing
      const int slot_x = other_half(slot, half);
      const int qa = base + sl, qb = qa + CHUNK;  // the staged columns of chunks c, c + 1
      const int col_o = slot * nvar + var_of(qo);
      const int col_a = (half ? slot_x : slot) * nvar + var_of(qa);
      f32x4 g[VH / 2];
      gather_bg(col_a, g);
      const bool nog = CWBL_DBG_STOP(c) == 13;  // (timing ablation, see gather_bg)
      const uint8_t okb = nog ? 1 : gld(T.col_ok, (unsigned)col_o);
      const float err = nog ? 1.0f : gld(T.col_err, (unsigned)col_o);
      const float omm = nog ? 0.0f : gld(T.col_omm, (unsigned)col_o);
      const f32x4 rd = nog ? f32x4{0.0f, 0.0f, 0.0f, 0.0f}
                           : gld4(reinterpret_cast<const float *>(T.rdata), 4u * (unsigned)slot);
      const bool ok = qo < npairs && okb != 0;
      const float wv =
          error_inv(c.weight_function, err, slot_r2(rd, T.tree_dim, q0, q1, q2), ch.expt);
      const float w = ok ? wv : 0.0f;
      const float yo = ok ? omm * wv : 0.0f;  // omm * error_inv (:451)
      ptot += __popcll(__ballot(ok));
      const float w_x = other_half(w, half);
      // chunk c + 1's staged column and weight, formed now: four values (col_b, w_b, yo,
      // slot_next) stay live across chunk c's accumulation
      const int col_b = (half ? slot : slot_x) * nvar + var_of(qb);
      const float w_b = half ? w : w_x;
      if (half == 0) {
        ch.yo[sl] = yo;
        if constexpr (PITCH > KP) ch.at(sl, KP) = yo;
        side.yo(sl, yo);
      }
      put(g, half ? w_x : w);
      side.stage(half, sl, g, half ? w_x : w);
      const bool two = base + CHUNK < npairs;  // wave-uniform
      if (two) gather_bg(col_b, g);  // chunk c + 1's bg rows in flight during chunk c's MFMAs
      __syncthreads();
      accumulate(min(CHUNK, npairs - base));
      __syncthreads();
      if (two) {
        if (half == 1) {
          ch.yo[sl] = yo;
          if constexpr (PITCH > KP) ch.at(sl, KP) = yo;
          side.yo(sl, yo);
        }
        put(g, w_b);
        side.stage(half, sl, g, w_b);
        __syncthreads();
        accumulate(min(CHUNK, npairs - base - CHUNK));
        __syncthreads();
      }
    }
  }
  return ptot;
}

// stage_columns for the 256-thread kernels (analysis path) with two chunk buffers: the
// gathers of chunk c + 1 are issued before chunk c is accumulated and committed (weights,
// LDS writes) to the other buffer after it, so their latency hides behind the matrix cores;
// one barrier per chunk.  Same columns, order and arithmetic as stage_columns;
// accumulate(nsl, chunk) reads the chunk to accumulate.
template <int KP, int CHUNK, int NT, bool XSW, class Acc>
__device__ __forceinline__ int stage_columns_pipe(
    ColumnChunk<KP, CHUNK, float, KP, false, XSW> (&ch)[2], const TreeDesc *__restrict__ trees, const SolveConsts &c,
    int gi, int lane, const int *__restrict__ nbr_cnt, const int *__restrict__ nbr_idx,
    const float3 pt, Acc &&accumulate) {
  static_assert(NT > 64 && NT % CHUNK == 0 && CHUNK <= 64, "threads per staged column");
  constexpr int LPC = NT / CHUNK;     // threads per staged column
  constexpr int VH = KP / (2 * LPC);  // float2 of the bg row per thread
  static_assert(KP % (4 * LPC) == 0, "bg row split into 16-B loads");
  int ptot = 0;
  if (lane < 32) ch[0].expt[lane] = kExpT[lane];
  __syncthreads();  // (LDS is not cleared between workgroups)
  const int sl = lane % CHUNK, half = lane / CHUNK;
  // XSW: a thread gathers and stores its VH / 2 float4 of the bg row starting at float4
  // (sl >> 1) mod VH / 2, so the 16 threads of a store group write 8 row offsets (with the
  // odd columns' r ^ 16 on top) instead of one
  static_assert(!XSW || ((VH / 2) & (VH / 2 - 1)) == 0, "rotation modulo a power of two");
  const int rot = XSW ? (sl >> 1) & (VH / 2 - 1) : 0;
  int cur = 0;
  for (int t = 0; t < c.ntrees; ++t) {
    const TreeDesc T = trees[t];
    const float q0 = pt.x * T.hclr_inv, q1 = pt.y * T.hclr_inv;  // get_lz (:243-253)
    const float q2 = T.query3d ? pt.z * T.vclr_inv : 0.0f;
    const int cnt = gptr(nbr_cnt)[(long long)gi * c.ntrees + t];
    const int nvar = T.nvar;
    const int npairs = cnt * nvar;
    if (npairs == 0) continue;
    const int *__restrict__ lst = nbr_idx + list_index(gi, c.list_cap, T.list_off);
    const float rnv = 1.0f / (float)nvar;
    auto divn = [&](int q) {
      if (nvar == 1) return q;
      int j = (int)((float)q * rnv);
      j -= j * nvar > q ? 1 : 0;
      j += (j + 1) * nvar <= q ? 1 : 0;
      return j;
    };
    auto slot_of = [&](int base) {  // this lane's slot of the chunk at base (0 past the list)
      return sl < min(CHUNK, npairs - base) ? gld(lst, list_slot(divn(base + sl))) : 0;
    };
    struct Gath {
      f32x4 g[VH / 2];
      f32x4 rd;
      float err, omm;
      uint8_t okb;
      bool live;
    };
    auto gather = [&](int base, int slot, Gath &G) {
      G.live = sl < min(CHUNK, npairs - base);
      if (CWBL_DBG_STOP(c) == 13) {  // timing ablation: the assembly without the gathers
#pragma unroll
        for (int i = 0; i < VH / 2; ++i) G.g[i] = f32x4{1.0f, 1.0f, 1.0f, 1.0f};
        G.rd = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        G.err = 1.0f;
        G.omm = 0.0f;
        G.okb = 1;
        return;
      }
      const int q = base + sl;
      const int jn = divn(q), v = q - jn * nvar;
      const int col = slot * nvar + v;  // a valid table index even past the list (slot 0)
      const unsigned b0 = (unsigned)(col * KP + 2 * VH * half);
#pragma unroll
      for (int i = 0; i < VH / 2; ++i)
        G.g[i] = gld4(T.col_bg, b0 + 4u * (unsigned)((i + rot) & (VH / 2 - 1)));
      G.okb = gld(T.col_ok, (unsigned)col);
      G.err = gld(T.col_err, (unsigned)col);
      G.omm = gld(T.col_omm, (unsigned)col);
      G.rd = gld4(reinterpret_cast<const float *>(T.rdata), 4u * (unsigned)slot);
    };
    auto commit = [&](const Gath &G, ColumnChunk<KP, CHUNK, float, KP, false, XSW> &dst) {
      // Every gathered register is consumed here, unconditionally: a dead component (rd.w)
      // would have its register reused at once, and a use the compiler sinks into a divergent
      // branch leaves the load pending on the skipping path; either way a later write to
      // the register waits for the load (vmcnt) and the gathers no longer overlap the MFMAs.
#pragma unroll
      for (int i = 0; i < VH / 2; ++i) asm volatile("" ::"v"(G.g[i]));
      asm volatile("" ::"v"(G.rd), "v"(G.err), "v"(G.omm), "v"((int)G.okb));
      const bool ok = G.live && G.okb != 0;
      const float wv =
          error_inv(c.weight_function, G.err, slot_r2(G.rd, T.tree_dim, q0, q1, q2), ch[0].expt);
      const float w = ok ? wv : 0.0f;
      const float yo = ok ? G.omm * wv : 0.0f;  // omm * error_inv (:451)
      ptot += __popcll(__ballot(ok && half == 0));  // counted by wave 0
      if (half == 0) dst.yo[sl] = yo;
#pragma unroll
      for (int i = 0; i < VH / 2; ++i) {  // bg * error_inv (:452)
        const int r = 2 * VH * half + 4 * ((i + rot) & (VH / 2 - 1));
        *reinterpret_cast<float2 *>(&dst.at(sl, r)) = make_float2(G.g[i].x * w, G.g[i].y * w);
        *reinterpret_cast<float2 *>(&dst.at(sl, r + 2)) = make_float2(G.g[i].z * w, G.g[i].w * w);
      }
    };
    int slot_n = slot_of(CHUNK);  // chunk 1's slots, loaded behind chunk 0's gathers
    {
      Gath G;
      gather(0, slot_of(0), G);
      commit(G, ch[cur]);
    }
    __syncthreads();
    for (int base = 0; base < npairs; base += CHUNK) {
      const int nsl = min(CHUNK, npairs - base);
      const int nb = base + CHUNK;
      Gath Gn;
      int slot_nn = 0;
      if (nb < npairs) {  // wave-uniform
        gather(nb, slot_n, Gn);
        slot_nn = slot_of(nb + CHUNK);
      }
      accumulate(nsl, ch[cur]);
      if (nb < npairs) commit(Gn, ch[cur ^ 1]);
      __syncthreads();  // chunk cur ^ 1 is written; everyone is done reading chunk cur
      cur ^= 1;
      slot_n = slot_nn;
    }
  }
  return ptot;
}

// Column assembly on the VALU: thread L accumulates the 4x4 blocks L, L+NT, ... of the lower
// block triangle of Yb Yb^T, and threads < KP the entries of Yb d.
template <int KP, int CHUNK, bool ASSEMBLED, int NT = 64, class E = float>
__device__ __forceinline__ void assemble_point(
    ColumnChunk<KP, CHUNK, E> &ch, const TreeDesc *__restrict__ trees, const SolveConsts &c,
    int gi, int lane, const int *__restrict__ nbr_cnt, const int *__restrict__ nbr_idx,
    const float3 pt, const long long *__restrict__ col_off,
    const float *__restrict__ yo_in, const float *__restrict__ yb_in,
    const int (&bi)[AsmLayout<KP, NT>::NBL], const int (&bj)[AsmLayout<KP, NT>::NBL],
    double (&acc)[AsmLayout<KP, NT>::NBL][16], double &b1acc, int &ptot) {
  constexpr int NBL = AsmLayout<KP, NT>::NBL, NBLK = AsmLayout<KP, NT>::NBLK;
#pragma unroll
  for (int it = 0; it < NBL; ++it)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[it][e] = 0.0;
  b1acc = 0.0;
  ptot = stage_columns<KP, CHUNK, ASSEMBLED, NT, E>(
      ch, trees, c, gi, lane, nbr_cnt, nbr_idx, pt, col_off, yo_in, yb_in, [&](int nsl) {
        for (int s = 0; s < nsl; ++s) {
#pragma unroll
          for (int it = 0; it < NBL; ++it) {
            if (lane + NT * it < NBLK) {
              double a4[4], b4[4];
              if constexpr (sizeof(E) == 8) {
                const double2 a0 = *reinterpret_cast<const double2 *>(&ch.yb[s][4 * bi[it]]);
                const double2 a1 = *reinterpret_cast<const double2 *>(&ch.yb[s][4 * bi[it] + 2]);
                const double2 c0 = *reinterpret_cast<const double2 *>(&ch.yb[s][4 * bj[it]]);
                const double2 c1 = *reinterpret_cast<const double2 *>(&ch.yb[s][4 * bj[it] + 2]);
                a4[0] = a0.x; a4[1] = a0.y; a4[2] = a1.x; a4[3] = a1.y;
                b4[0] = c0.x; b4[1] = c0.y; b4[2] = c1.x; b4[3] = c1.y;
              } else {
                const float4 ra = *reinterpret_cast<const float4 *>(&ch.yb[s][4 * bi[it]]);
                const float4 rb = *reinterpret_cast<const float4 *>(&ch.yb[s][4 * bj[it]]);
                a4[0] = ra.x; a4[1] = ra.y; a4[2] = ra.z; a4[3] = ra.w;
                b4[0] = rb.x; b4[1] = rb.y; b4[2] = rb.z; b4[3] = rb.w;
              }
#pragma unroll
              for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  acc[it][4 * r + q] = fma(a4[r], b4[q], acc[it][4 * r + q]);
            }
          }
          if (lane < KP) b1acc = fma((double)ch.yb[s][lane], (double)ch.yo[s], b1acc);
        }
      });
}

// Column assembly on the matrix cores (v_mfma_f64_16x16x4_f64): Y' = [Yb; yo] padded to
// 16*NT rows, and the lower tiles (I >= J) of Y' Y'^T accumulate in registers
// (C/D map: col = lane&15, row = (lane>>4) + 4*reg).  Row KP of Y' is yo when it fits in
// the padding (YO_ROW), so row KP of the product is Yb d; otherwise Yb d is summed on the
// VALU by lanes < KP.  Products of fp32 values are exact in fp64 and every tile is a
// sequence of fp64 fused multiply-adds, like the dsyrk of the reference.
//
// The last tile row holds only KP+1-16(NT-1) live rows (9 at KP = 40: rows 32..39 and yo).
// With SPLIT_LAST its tiles are not 16x16 products but NBL4 < 4 four-row strips, one
// v_mfma_f64_4x4x4f64 each (16 cycles instead of 64 for the whole tile): its 4 blocks b
// compute rows 4r..4r+3 of the strip against rows 4b..4b+3 of tile column J, with the strip
// rows broadcast to every block (A lane 16k+4b+i = Y'[16(NT-1)+4r+i][k]) and tile column J
// as B in the 16x16 operand layout itself (B lane 16k+4b+j = Y'[16J+4b+j][k]).  Its result
// lane 16i+4b+j = (row 16(NT-1)+4r+i, col 16J+4b+j) is register r of the 16x16 tile's C/D
// map, so the strips accumulate straight into tile registers 0..NBL4-1 (register 3 stays
// zero: rows past yo).  At KP = 40: 9 strip MFMAs x 16 cycles instead of 3 tiles x 64 per 4
// columns, 336 matrix-pipe cycles per 4 columns instead of 384.
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int KP>
struct MfmaLayout {
  static constexpr int NT = (KP + 15) / 16;              // 16-row tiles per dimension
  static constexpr bool YO_ROW = KP + 1 <= 16 * NT;      // yo rides in the padding
  static constexpr int NTL = NT * (NT + 1) / 2;          // lower tiles
  static constexpr int PITCH = YO_ROW ? 16 * NT : KP;    // staged column length
  static constexpr bool SWZ = PITCH % 32 == 16;          // shifted columns (ColumnChunk)
  static constexpr bool XSW = PITCH % 32 == 0;           // odd columns' rows ^ 16 (ColumnChunk)
  static constexpr int NBL4 = YO_ROW ? (KP + 1 - 16 * (NT - 1) + 3) / 4 : 4;  // live strips
  static constexpr bool SPLIT_LAST = NBL4 < 4;
};

template <int KP, int CHUNK, bool ASSEMBLED>
__device__ __forceinline__ void assemble_point_mfma(
    ColumnChunk<KP, CHUNK, float, MfmaLayout<KP>::PITCH, MfmaLayout<KP>::SWZ,
                MfmaLayout<KP>::XSW> &ch,
    const TreeDesc *__restrict__ trees,
    const SolveConsts &c, int gi, int lane, const int *__restrict__ nbr_cnt,
    const int *__restrict__ nbr_idx, const float3 pt, const long long *__restrict__ col_off,
    const float *__restrict__ yo_in, const float *__restrict__ yb_in,
    f64x4 (&tile)[MfmaLayout<KP>::NTL], double &b1acc, int &ptot) {
  using L = MfmaLayout<KP>;
#pragma unroll
  for (int t = 0; t < L::NTL; ++t) tile[t] = f64x4{0.0, 0.0, 0.0, 0.0};
  b1acc = 0.0;
  const int kk = lane >> 4, m = lane & 15;
  auto stage = [&](auto &&acc) {
    if constexpr (!ASSEMBLED && CHUNK == 32)
      return stage_columns_pair<KP, CHUNK, MfmaLayout<KP>::PITCH, MfmaLayout<KP>::SWZ>(
          ch, trees, c, gi, lane, nbr_cnt, nbr_idx, pt, acc);
    else
      return stage_columns<KP, CHUNK, ASSEMBLED>(ch, trees, c, gi, lane, nbr_cnt, nbr_idx, pt,
                                                 col_off, yo_in, yb_in, acc);
  };
  ptot = stage([&](int nsl) {
        // Column s = 4 g + kk of the chunk feeds k-slot kk of group g; every staged column
        // past nsl is zero (stage_columns writes the whole chunk), and with YO_ROW the
        // staged rows are [Yb; yo; 0] up to 16 NT, so the operand reads need no predicate.
        // The group loop is unrolled (immediate LDS offsets, static double buffer), and the
        // next group's reads are issued before this group's MFMAs, so the LDS latency hides
        // behind the matrix pipe.
        static_assert(CHUNK % 4 == 0, "k-slots");
        constexpr int NS = L::SPLIT_LAST ? L::NBL4 : 1;
        float f[2][L::NT], fy[2], fs[2][NS];
        const float *c0 = ch.col(kk);  // column 4 g + kk at c0 + g GSTRIDE
        const int xk = ch.xr(kk);      // (XSW: the rows of an odd column are r ^ 16)
        auto load = [&](int b, int g) {
          const float *cs = c0 + g * ch.GSTRIDE;
#pragma unroll
          for (int I = 0; I < L::NT; ++I) {
            const int row = 16 * I + m;
            if constexpr (L::YO_ROW) f[b][I] = cs[row ^ xk];
            else f[b][I] = cs[(row < KP ? row : KP - 1) ^ xk];
          }
          if constexpr (L::SPLIT_LAST) {  // strip rows, broadcast over the 4 blocks
#pragma unroll
            for (int r = 0; r < NS; ++r) fs[b][r] = cs[(16 * (L::NT - 1) + 4 * r + (m & 3)) ^ xk];
          }
          if constexpr (!L::YO_ROW) fy[b] = ch.yo[4 * g + kk];
        };
        const int nl = CWBL_DBG_STOP(c) == 11 ? 0 : nsl;
        if (nl > 0) load(0, 0);
#pragma unroll
        for (int g = 0; g < CHUNK / 4; ++g) {
          if (4 * g >= nl) break;  // nsl is wave-uniform
          const int b = g & 1;
          double op[L::NT];
#pragma unroll
          for (int I = 0; I < L::NT; ++I) {
            if constexpr (L::YO_ROW) {
              op[I] = (double)f[b][I];
            } else {
              const int row = 16 * I + m;
              op[I] = (double)(row < KP ? f[b][I] : 0.0f);
            }
          }
          double os[NS];
#pragma unroll
          for (int r = 0; r < NS; ++r) os[r] = L::SPLIT_LAST ? (double)fs[b][r] : 0.0;
          if (g + 1 < CHUNK / 4 && 4 * (g + 1) < nl) load(b ^ 1, g + 1);
          int t = 0;
#pragma unroll
          for (int I = 0; I < L::NT; ++I)
#pragma unroll
            for (int J = 0; J <= I; ++J, ++t) {
              if (L::SPLIT_LAST && I == L::NT - 1) {
#pragma unroll
                for (int r = 0; r < NS; ++r)
                  tile[t][r] = __builtin_amdgcn_mfma_f64_4x4x4f64(os[r], op[J], tile[t][r], 0, 0, 0);
              } else {
                tile[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(op[I], op[J], tile[t], 0, 0, 0);
              }
            }
        }
        if constexpr (!L::YO_ROW) {
          for (int s = 0; s < nsl; ++s)
            if (lane < KP) b1acc = fma((double)ch.at(s, lane), (double)ch.yo[s], b1acc);
        }
      });
}

// thread -> 4x4 block (bi, bj) of the lower block triangle, row-major over the triangle
template <int KP, int NT = 64>
__device__ __forceinline__ void block_of_lane(int lane, int (&bi)[AsmLayout<KP, NT>::NBL],
                                              int (&bj)[AsmLayout<KP, NT>::NBL]) {
#pragma unroll
  for (int it = 0; it < AsmLayout<KP, NT>::NBL; ++it) {
    const int b = lane + NT * it;
    int rr = 0;
    while ((rr + 1) * (rr + 2) / 2 <= b) ++rr;
    bi[it] = rr;
    bj[it] = b - rr * (rr + 1) / 2;
  }
}

}  // namespace cwbl
