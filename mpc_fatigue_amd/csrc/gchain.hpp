// The C2 chain family's kernels (csrc/gchain.hip): what the generic solver's host loop (gipm.hip) calls.
#pragma once
#include "gcore.hpp"

namespace mf {

// Pilz chain, 6 joints, one end-effector frame, the two line rows, no thermal states: the family of the C2 / C5 batch
using ChainC2 = ChainFam<6, 1, 2, false>;
// families with explicit Euler dynamics and line rows that k_gkkt_chain takes
template <class FAM> struct ChainEuler { static constexpr bool value = false; };
template <> struct ChainEuler<ChainC2> { static constexpr bool value = true; };

// k_geval_chain<ChainC2, 0 / 1> (the q and the qd directions), blocks = 8 NJ ceil(ceil(batch N / 64) / 8)
void gchain_eval(hipStream_t s, int blocks, const DevModel *M0, const DevFrame *F0, const GParams &P, const GArrays &A,
                 int batch);
// k_gkkt_chain<ChainC2>, one wavefront per horizon (horizons of at most GCHAIN_NMAX stages)
constexpr int GCHAIN_NMAX = 1024;
void gchain_kkt(hipStream_t s, const GParams &P, const GArrays &A, int batch);

}  // namespace mf
