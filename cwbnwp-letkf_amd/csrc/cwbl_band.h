// cwbl_band.h — shared by the two-stage kernels (cwbl_band.hip: band_head_kernel,
// cwbl_band_tail.hip: band_tail_kernel): DPP helpers, the workspace record, the chase plan.
#pragma once
#include "cwbl_device.h"


#include <type_traits>
#include <utility>

namespace cwbl {

namespace band_detail {


// value of lane L of this lane's 16-lane row (DPP row_newbcast, one v_mov_b64)
template <int L>
__device__ __forceinline__ double rbcast(double x) {
  return __longlong_as_double(
      __builtin_amdgcn_update_dpp(0ll, __double_as_longlong(x), 0x150 + L, 0xf, 0xf, true));
}
// acc + x_L y and acc - x_L y, x_L = lane L of this lane's 16-lane row: one v_fmac_f64_dpp
// row_newbcast (gfx950's 64-bit DPP).  A DPP source must not be written by the VALU in the two
// instructions before: the callers write their sources once and pin them (dpp_pin, s_nop 1).
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

}  // namespace band_detail
using namespace band_detail;

// ---- the workspace record of one point ------------------------------------------------------
struct BandRec {
  static constexpr int N = 128, B = 8, NP = 15, NTASK = 1056;
  static constexpr int BAND = 0;                // [N][B+1]: A(i, i-d), d = 0..B
  static constexpr int U1 = BAND + N * (B + 1);   // Q1^T b1
  static constexpr int U2 = U1 + N;               // Q1^T x'
  static constexpr int PV = U2 + N;               // panel p: V (m_p x 8 row-major), m_p = 120-8p
  static constexpr int PT = PV + 8 * 960;         // panel p: T (8 x 8, upper)
  static constexpr int R2 = PT + NP * 64;         // chase reflector q: [q][0] tau, [q][e] v_e
  static constexpr int WORDS = R2 + NTASK * 8;
  __host__ __device__ static constexpr int pv(int p) { return PV + 8 * (120 * p - 4 * p * (p - 1)); }
};
static_assert(BandRec::pv(15) == BandRec::PT, "panel reflector offsets");

// the chase schedule (scripts/two_stage_b8.py: schedule): tasks of sweep j, their first index,
// and the round in which sweep j starts (two slots, sweep j+1 three tasks behind sweep j)
struct ChasePlan {
  int start[126], first[127], ntask[126];  // 32-bit: scalar loads
  int rounds;
};
__host__ __device__ constexpr int chase_ntask(int j) { return j <= 125 ? (125 - j) / 8 + 1 : 0; }
__host__ __device__ constexpr ChasePlan make_chase_plan() {
  ChasePlan p{};
  int acc = 0, end = 0;
  for (int j = 0; j < 126; ++j) {
    int s = 0;
    if (j >= 1 && p.start[j - 1] + 3 > s) s = p.start[j - 1] + 3;
    if (j >= 2 && p.start[j - 2] + p.ntask[j - 2] > s) s = p.start[j - 2] + p.ntask[j - 2];
    p.start[j] = s;
    p.ntask[j] = chase_ntask(j);
    p.first[j] = acc;
    acc += p.ntask[j];
    if (s + p.ntask[j] > end) end = s + p.ntask[j];
  }
  p.first[126] = acc;
  p.rounds = end;
  return p;
}
constexpr ChasePlan kChase = make_chase_plan();
static_assert(kChase.first[126] == BandRec::NTASK && kChase.rounds == 586, "chase plan");

}  // namespace cwbl
