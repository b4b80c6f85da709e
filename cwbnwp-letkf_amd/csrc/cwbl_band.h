// cwbl_band.h — shared by the two-stage kernels (cwbl_band.hip: band_head_kernel,
// cwbl_band_tail.hip: band_tail_kernel): the workspace record and the chase plan (the DPP
// row helpers are in cwbl_device.h).
#pragma once
#include "cwbl_device.h"

#include <type_traits>
#include <utility>

namespace cwbl {

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
