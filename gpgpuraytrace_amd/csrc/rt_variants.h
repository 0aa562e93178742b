// rt_variants.h -- compile-time knobs and diagnostic hooks of the trace kernels.
//
// The product build takes every default below.  A/B builds override a knob on the compiler line
// (`make -C gpgpuraytrace_amd/csrc variant NAME=x FLAGS="-DRT_LONG_BATCH=96"`, loaded by
// scripts/with_variant.py); diagnostic builds define one of the RT_DIAG_* switches at the end.  The
// kernel source (rt_kernels.hip) only names the constants and the one-line hooks, so the hot file
// reads as the product.  DESIGN.md sections 4-5 record what each knob measured.
#pragma once

// ---- k_trace's scheduler ----------------------------------------------------------------------
// near the unit queue's end (a wave took one of its last RT_NEAR_UNITS x wave-slots units; 0: off) the block
// takes long rays from RT_NEAR_LONG_BATCH queued instead of RT_LONG_BATCH: the blocks' long-ray backlog at
// the drain (p50 35 -> 10 rays at N = 8) and the N = 8 shard simulation -1.2%, N = 1 within noise
// (profiles/r05/tail_ab.md)
#ifndef RT_NEAR_UNITS
#define RT_NEAR_UNITS 2
#endif
#ifndef RT_NEAR_LONG_BATCH
#define RT_NEAR_LONG_BATCH 16
#endif
// (A/B) s_setprio of a long-ray wave once the near-end mode is on (0: off; a unit resets it to 0).  2: the N = 8
// shard simulation and bench within noise, the post-drain tail unchanged (profiles/r06/dpp_ab.md)
#ifndef RT_LONG_PRIO
#define RT_LONG_PRIO 0
#endif
// lanes idle before a long-ray wave refills them from the ring (amortises the refill's prologue)
#ifndef RT_REFILL_IDLE
#define RT_REFILL_IDLE 4
#endif
// the gated launch's prepass tasks: 0 = taken from a counter by whichever waves come first, 1 = each wave's by
// its first-unit index (one task wave per SIMD in block start order; measured slower: profiles/r05/gated_ab.md)
#ifndef RT_GATE_STATIC
#define RT_GATE_STATIC 0
#endif
// the gated launch: s_sleep argument (x 64 cycles) of a wave whose tile scan step found nothing ready
#ifndef RT_GATE_SLEEP
#define RT_GATE_SLEEP 0
#endif
// queued long rays that make a wave switch to them
#ifndef RT_LONG_BATCH
#define RT_LONG_BATCH 128
#endif
// live lanes below which a long-ray wave whose ring ran dry hands its rays back
#ifndef RT_COMPACT_LIVE
#define RT_COMPACT_LIVE 56
#endif
// after the unit queue drains (nomadplains): a long-ray wave with <= RT_SEG_HANDBACK live rays and an
// empty ring hands them back; a wave that finds <= RT_SEG_QUEUE queued marches them as segments of
// RT_SEG_LANES lanes per ray (0: off).  Round 5: 64 / 4096 (every post-drain wave with an empty ring
// hands back, every post-drain long-ray job is a segment job): the blocks' median post-drain tail -10%,
// the N = 8 shard simulation -0.3 to -1.6%, N = 1 within noise (profiles/r05/tail_ab.md; round 4: 16 / 64)
#ifndef RT_SEG_LANES
#define RT_SEG_LANES 8
#endif
#ifndef RT_SEG_HANDBACK
#define RT_SEG_HANDBACK 64
#endif
#ifndef RT_SEG_QUEUE
#define RT_SEG_QUEUE 4096
#endif
// 1: the octave-parallel density of the segment marches (not the LOWREG primary tail) evaluates all its
// rounds without a branch between them, so their LDS round trips overlap (latency-bound tail steps)
#ifndef RT_SEG_ILP
#define RT_SEG_ILP 0
#endif
// 1: density_nomadplains_seg with LPR <= 16 (k_trace's segment marches, primary tail and prepass tasks) sums
// the octaves on the segment's first lane from DPP row shifts and broadcasts the density (DPP); 0: every lane
// gathers the 18 values with ds_bpermute (through the LDS pipe)
#ifndef RT_SEG_DPP
#define RT_SEG_DPP 1
#endif
// 1: after the drain a long-ray wave refills nothing and hands back all its rays, so every post-drain long
// ray marches on a segment (with RT_SEG_QUEUE large enough that waves take them as segments)
#ifndef RT_SEG_DRAIN_ALL
#define RT_SEG_DRAIN_ALL 0
#endif
// a primary unit's last <= RT_PRIMARY_SEG rays march on 64 / RT_PRIMARY_SEG lanes each (0, 4, 8, 16)
#ifndef RT_PRIMARY_SEG
#define RT_PRIMARY_SEG 8
#endif
// AO counter slots per k_trace block in LDS (AO_SAMPLES >= 2; 0: device atomics count)
#ifndef RT_AO_SLOTS
#define RT_AO_SLOTS 256
#endif
// the instrumented (STATS) kernels take the product's primary segment tail too (1), so their march and
// noise counts are asserted through the timed kernel's code path; 0 keeps a 64-lane tail there
#ifndef RT_STATS_PRIMARY_SEG
#define RT_STATS_PRIMARY_SEG 1
#endif
// waves per k_trace block: 16 for the landscapes that fit 128 VGPRs, 12 for simple / greenrocks
#ifndef RT_TRACE_WAVES_FAST
#define RT_TRACE_WAVES_FAST 16
#endif
#ifndef RT_TRACE_WAVES_WIDE
#define RT_TRACE_WAVES_WIDE 12
#endif
// lane slots of the LDS gradient planes (rt_shader.h NoiseView): 16 makes the gxy ds_read_b128 reads
// conflict-free and the gz ds_read_b64 reads 2-way; 8 / 4 (every slot holds the same data, so the
// results are the same bits) double / quadruple both -- the A/B that prices the LDS bank conflicts
#ifndef RT_LDS_SLOTS
#define RT_LDS_SLOTS 16
#endif
// nomadplains FBM octave constants: 1 = scalar loads from the launch's constant block (every lane in
// the octave loop is at the same octave), 0 = a ds_read_b128 of the LDS octave table per octave.  The
// scalar form takes 4 of ~40 LDS-array cycles per octave off the CU's LDS (62% busy on k_trace):
// +1.0% Mray/s same box (profiles/r04/oct_smem_ab.txt)
#ifndef RT_OCT_SMEM
#define RT_OCT_SMEM 1
#endif
// (A/B) the SMEM octave loop's exit: 1 = a v_cmp of the scalar octave index against each lane's count, 53 VALU
// per octave instead of 54 (no per-lane countdown).  Bit-exact, measured within noise: 1505.4 / 1504.3 / 1475.9
// against 1505.2 / 1503.3 / 1504.2 Mray/s, alternating on one box (profiles/r06/oct_exit_ab.txt)
#ifndef RT_OCT_SCALAR_EXIT
#define RT_OCT_SCALAR_EXIT 0
#endif
// wave priority (s_setprio) of a fused prepass task (FusedPrepass) while it marches
#ifndef RT_FUSE_PRIO
#define RT_FUSE_PRIO 3
#endif
// k_order: RT_ORDER_BATCH forces the batch-wide (1) or frame-major (0) unit order; -1 = automatic
// (batch-wide below kOrderBatchUnitsPerWave units per wave slot)
#ifndef RT_ORDER_BATCH
#define RT_ORDER_BATCH -1
#endif

// UnitMap::fit with one AO ray: 1 = a hit's long shadow and its AO ray race for its pixel (device atomic OR on
// its aocc byte, the second stores it) and no k_finish runs; 0 = k_finish finishes those hits.  A/B only:
// bit-exact (all GPU tests), but HBM 3.44x -> 5.38x the RGBA8 frame and 1.0% slower same box
// (profiles/r06/fit_race_ab.md)
#ifndef RT_FIT_RACE
#define RT_FIT_RACE 0
#endif

// threads per block of a one-frame (and two-frame) camerarays prepass (RT_PREPASS_LPR1 lanes per ray; one block per
// CU, as it holds the noise tables).  A serial frame's prepass runs in the previous trace's tail, where CUs free one
// by one: fewer, larger blocks can start sooner, but 32 rays to a CU march slower than 8 or 16
#ifndef RT_PREPASS_BS1
#define RT_PREPASS_BS1 256
#endif
// lanes per ray of that prepass (32: one noise round per step and ds_bpermute gathers; 16 / 8: 2 / 3 rounds and
// the DPP sum, RT_SEG_DPP).  16 lanes (16 rays a block, 64 blocks): the serial frame loop 3.369 -> 3.311 ms per
// frame same box (4 runs each; 8 lanes / 128 blocks and 16 lanes / 32 blocks slower; profiles/r06/dpp_ab.md)
#ifndef RT_PREPASS_LPR1
#define RT_PREPASS_LPR1 16
#endif

// (A/B) noise3d's z-layer replication t + Z * 0x01010101 as an inline v_mad_u32_u24
#ifndef RT_Z_MAD24
#define RT_Z_MAD24 0
#endif

// AO generator records (AO_SAMPLES >= 2): a hit's AO rays as one ring record expanded at refill (A/B only:
// bit-exact, C5 HBM 5.9x -> 5.0x but 24% slower; profiles/r05/ao_gen_ab.md)
#ifndef RT_AO_GEN
#define RT_AO_GEN 0
#endif
// RT_FBM_EXIT=K (A/B only, 0 in the product): the exact FBM early exit of the primary march.  After K
// octaves a sample whose density provably stays in the unit-step no-hit band [-5, 0) (the remaining
// octaves' amplitude bound from the LDS octave table's prefix column) skips the
// rest; a sample after which the march could exit is always exact.  profiles/r05/fbm_exit_ab.md.
#ifndef RT_FBM_EXIT
#define RT_FBM_EXIT 0
#endif

// ---- diagnostic builds (never in the product) ------------------------------------------------
// RT_WAVE_TRACE          per-wave timeline of k_trace (make trace; scripts/wave_trace.py); fields 23-27: segment-job
//                        time / jobs / loop steps, lane-refill long-ray loop steps / time
// RT_LIVE_HIST           histogram of live lanes per primary march step (rt_debug_live_hist)
// RT_COUNT_PRIMARY_STEPS count live lanes per primary march step as noise (scripts/phase_util.py)
// RT_COUNT_LONG_STEPS=k  the same for long-ray steps (1 always, 2 after the drain, 3 before)
// RT_COUNT_PHASE=k       count only the noise of k_trace work kind k (rt_shader.h count_noise)
// RT_EXTRA_OCTAVE=n      n dead octaves per nomadplains density sample (issue-cost experiment)
// RT_DIAG_SKIP=mask      HBM attribution: drop a class of stores (wrong pixels, same control flow):
//                        1 miss pixels, 2 k_trace hit pixels (fit), 4 hit samples, 8 AO-count atomics,
//                        16 long-shadow fin records, 64 k_finish pixels
#ifndef RT_DIAG_SKIP
#define RT_DIAG_SKIP 0
#endif
// RT_DIAG_HITPAD=1        fog-free hit records padded from 16 to 32 B (the hit stack's HBM write cost)
#ifndef RT_DIAG_HITPAD
#define RT_DIAG_HITPAD 0
#endif
#ifdef RT_WAVE_TRACE
#define RT_WT_FIELDS 28
#define RT_WT_MAX_WAVES 8192
#define WT(...) __VA_ARGS__
#else
#define WT(...)
#endif
#ifdef RT_LIVE_HIST
#define RT_DIAG_LIVE_HIST(...) __VA_ARGS__
#else
#define RT_DIAG_LIVE_HIST(...)
#endif
#ifdef RT_COUNT_PRIMARY_STEPS
#define RT_DIAG_PRIMARY_STEPS(...) __VA_ARGS__
#else
#define RT_DIAG_PRIMARY_STEPS(...)
#endif
#ifdef RT_COUNT_LONG_STEPS
#define RT_DIAG_LONG_STEPS(...) __VA_ARGS__
#else
#define RT_DIAG_LONG_STEPS(...)
#endif
