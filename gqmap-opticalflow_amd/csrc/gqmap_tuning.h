// gqmap_tuning.h -- compile-time knobs of the HIP iteration kernels
// (gqmap_engine.hip).  None of them changes a result: every setting computes
// the same bits (the arithmetic is specified by gqmap_math.h); they choose
// unrolling, register budgets and kernel shapes.  The defaults are the
// measured best on MI355X (profiles/ named per knob).  A -D on
// the compiler line overrides one for an A/B build (scripts/ab_build.sh).
#pragma once

// Edge quadrature: mirror pairs per loop trip, fp64 and fp32 (r02_pair_unroll)
#ifndef GQ_EDGE_UNROLL_N
#define GQ_EDGE_UNROLL_N 2
#endif
#ifndef GQ_PAIR_UNROLL_N
#define GQ_PAIR_UNROLL_N 2
#endif
// ... at one lane per node for fp32 and the ctf levels (round 5,
// profiles/r05_unroll_knobs.txt: 4 gains 2.4% on C2 fp32 and 0.8% on the
// 480x640 level; fp64 C2 stays at 2)
#ifndef GQ_PAIR_UNROLL_Q1
#define GQ_PAIR_UNROLL_Q1 4
#endif
// Node quadrature: points per loop trip (r03_small_node_unroll: 1 is best)
#ifndef GQ_NODE_UNROLL_N
#define GQ_NODE_UNROLL_N 1
#endif
// Finalize: the NFIX fixed sums loaded together (fp32 C2 -2 us)
#ifndef GQ_FIN_GROUP
#define GQ_FIN_GROUP 1
#endif
// fp32: mirror-pair edge sums on packed float2 registers (r02_lane_mask_pk)
#ifndef GQ_EDGE_PK
#define GQ_EDGE_PK 1
#endif
// Q > 1: the quadrature table staged in LDS (lane-varying indices)
#ifndef GQ_TAB_LDS
#define GQ_TAB_LDS 1
#endif
// Co-resident workgroups alternate node-first / edge-first phase order
#ifndef GQ_PHASE_MIX
#define GQ_PHASE_MIX 1
#endif
// ... with the order flipped (co-resident blocks j, j+S, j+2S: edge, node,
// edge) on the ctf Q = 1 kernel (profiles/r05_phase_mix_inv.txt)
#ifndef GQ_PHASE_MIX_CTF_Q1_INV
#define GQ_PHASE_MIX_CTF_Q1_INV 1
#endif
#ifndef GQ_PHASE_MIX_OTHER_INV  // the other single-pixel kernels
#define GQ_PHASE_MIX_OTHER_INV 0
#endif
// Waves per SIMD the register allocation must allow (MI355X: 136-168 VGPRs
// -> 3, 176-256 -> 2).  Left to the allocator: forcing 3 waves on the
// single-scale engine moved arrays to scratch (C2 +24%); bounding the super
// engine to 2 made its block sum 25% slower than the allocator's own schedule.
#ifndef GQ_MIN_WAVES
#define GQ_MIN_WAVES 1
#endif
#ifndef GQ_SUPER_WAVES
#define GQ_SUPER_WAVES 1
#endif
#ifndef GQ_MIDQ_WAVES  // single-pixel engines at Q = 2, 4, 8
#define GQ_MIDQ_WAVES 1
#endif
// Smallest lanes-per-node split whose edge jobs prefetch the next job's
// operands / run fully unrolled (r02_edge_prefetch_ab)
#ifndef GQ_PREFETCH_MIN_Q
#define GQ_PREFETCH_MIN_Q 2
#endif
// Node quadrature software-pipelined (node_sums PF) from this many lanes per
// node up; 99 = never.  Round 5 (profiles/r05_node_pf_ab.txt): C2 fp64
// k_iter -1.3%, ctf 480x640 -0.5%, 388x75 strip -1%, 240x320 / 120x160
// unchanged, same bits; the C2 kernel at 164 VGPRs instead of 168.
#ifndef GQ_NODE_PF_MIN_Q
#define GQ_NODE_PF_MIN_Q 1
#endif
#ifndef GQ_UNROLL_MIN_Q
#define GQ_UNROLL_MIN_Q 2
#endif
// Persistent small-level launch: also at Q = 4 (r03_persist_levels: slower, off)
#ifndef GQ_PERSIST_Q4
#define GQ_PERSIST_Q4 0
#endif
// Persistent grid barrier: s_sleep between polls
#ifndef GQ_PERSIST_SLEEP
#define GQ_PERSIST_SLEEP 2
#endif
// Debug builds only: per-workgroup s_memrealtime stamps of k_iter iterations
// GQ_TIMELINE and GQ_TIMELINE + 1 (gqmap_debug_timeline, scripts/timeline.py)
#ifndef GQ_TIMELINE
#define GQ_TIMELINE 0
#endif
