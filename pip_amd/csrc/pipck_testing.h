/*
 * pipck_testing.h -- INTERNAL tuning hook of libpipck.so, for the GPU tests and
 * the measurement tools only (tests/, tools/).  Not part of the public ABI in
 * include/pipck.h: it is process-global mutable state that changes kernel
 * selection for every context and thread, so a product caller must never
 * use it.  Every setting computes the same results (the GPU tests sweep them
 * against the oracle); only speed changes -- except bit 21 below, a
 * measurement-only probe.  pipck_tune(0, 0, 0, 0) restores
 * the automatic choice.
 */
#ifndef PIPCK_TESTING_H
#define PIPCK_TESTING_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Launch-shape override for tuning; 0 = automatic everywhere (process-wide, internal).
 * lanes_per_packet in {1,2,4,8,16,32,64} and loads_per_lane pick the fixed
 * kernel's shape; lanes_per_packet = 256 selects k_wave (pipck_wave.hip: one
 * packet per wavefront, the north_star's sketch, a measurement arm) for fixed
 * strides and descriptor batches, loads_per_lane 2/4/8/16 its chunks per lane
 * per pass (loads_per_lane in {2,4,8} also sets the ragged kernel's rows
 * in flight; for the flat-stream kernel 2/4/8/16 rows, 3/5/9/13/17/25/33 =
 * ring-pipelined 2/4/8/12/16/24/32); blocks caps the grid; flags bit 0 = plain (cached) loads, bit 2 =
 * non-temporal loads (default: per kernel), bit 1 = never use the flat-stream
 * fixed kernel, bit 3 = XCD-grouped task split, bit 4 = no packed-tile
 * addressing in the ragged kernel, bit 5 = 4-wave ragged blocks (default 1),
 * bit 6 = never the small-packet kernel (packets <= 64 B incl. chunk offset),
 * bit 7 = never the short-stride flat kernel (16-B-multiple strides < 1 KiB),
 * bits 8..15 = 1 KiB rows per flat-kernel wave task (default 64), bit 16 = no
 * lane-per-segment path for ragged tiles of tiny segments, bit 17 = never the
 * tiny-stride flat kernel (8-B-multiple strides <= 64 B with pseudo-headers or
 * RX verify; loads_per_lane 4/8/16 = its ring, bits 8..15 its rows per wave
 * task, default 4 and 12), bit 18 = that kernel without pseudo-headers too, bits 24..27 =
 * small-kernel packets per lane (1 = 2, 2 = 4, 3 = 8, 4 = 16; default 2), bit 19 = mixed rows of
 * packed ragged tiles always find segments through LDS marks (default: a scalar
 * loop over up to 4 segment ends per row).  The packed-batch kernel
 * (pipck_checksum_packed) takes loads_per_lane 17/25/33 = a ring of 16/24/32.
 * The byte-packed kernels (pipck_checksum_packed_bytes, k_packedb, default 8
 * waves per tile with rings of 3; pipck_rx_verify_device, k_packedb_rx,
 * default 4 waves with rings of 8) take loads_per_lane 32 = one wave per tile
 * with a ring of 32 (the round-4 shape), 48 = 4 waves x 8, 72 / 74 = 8 waves
 * x 2 / 4 (k_packedb only), 28 = 2 waves x 16 (k_packedb_rx only).
 * Bit 20 = record the per-task timeline (pipck_trace_tasks below).
 * Bit 21 = MEASUREMENT ONLY, WRONG RESULTS: k_flat waits for and consumes every
 * row with one add and does no per-packet work (times the access pattern
 * alone).  Bit 22 = MEASUREMENT ONLY, NO RESULTS: k_flat skips its task end.
 * Bit 23 = MEASUREMENT ONLY, NO RESULTS: k_flat computes its results but stores
 * none (bits 21-23 isolate the task-end cost, profiles/r03_flat_end_probe.jsonl).
 * Bits 21-23 launch separate probe kernels (k_flat_probe, k_flat_coop_probe:
 * checksum mode, non-temporal loads, rings 24/32 for k_flat); the production
 * kernels have them compiled out and ignore them otherwise.
 * Bit 28 = the other fixed-stride schedule (and for pipck_rx_verify_ring the
 * row stream k_ring_rx instead of the default k_ring; lanes_per_packet = 256
 * there selects k_ring_slots, loads_per_lane 8 / 24 k_ring's loads in flight,
 * the blocks argument 8 / 16 / 32 makes its interleaved row stream cover so
 * many slots at a time; its other switches are pipck_tune_ring's, below):
 * k_flat (one task per wave)
 * instead of the block-cooperative k_flat_coop, the default for 16-B-multiple
 * strides from 1 KiB to 64 KiB except exactly 1 and 2 KiB (there the reverse);
 * for k_flat_coop, bits 8..15 are rows per wave
 * (default 48, jumbo 64) and loads_per_lane 17/25/33 its ring (default 32).  Bit 29 = result stores with the r02
 * write-back policy in k_flat / k_packed instead of write-through (sc1).
 * Bit 30 = the r02 schemes: per-wave result stores in k_flat (default: one
 * coalesced store per block), tile rows from the tile's first chunk in k_packed
 * (default: from its 128-B line).  Bit 31 = k_flat tasks of exactly the packet
 * count the rows knob gives (default: a multiple of 16 for strides < 4 KiB).
 * Bits 24..27 = the small kernel's depth (above).  Bits 29-31 compute the same
 * results; they exist for the separate-process A/Bs recorded in profiles/.
 * The header row kernel (k_hdr: 20/24-byte strides, no pseudo-header) takes
 * loads_per_lane 8/16/24/32 = its ring (default 32) and 1 = never k_hdr (k_small
 * instead), bits 8..15 = its rows per wave task, and reads bits 29-31 as its
 * result-store policy: 29 = plain write-back, 30 = non-temporal (default
 * write-through sc1), 31 = one store per result instead of 16-byte pieces. */
void pipck_tune(uint32_t lanes_per_packet, uint32_t loads_per_lane, uint32_t blocks, uint32_t flags);

/* MEASUREMENT-ONLY probes that CHANGE RESULTS, kept apart from pipck_tune's
 * flags (whose settings all compute the same results; process-wide, internal).
 * Bit 0 = k_hdr stores each IPv4 header's checksum into the header's ip_sum
 * (htons, byte 10, as pip_netif.cpp:97 stores it) and leaves the result array
 * untouched (the "results inside the headers" layout).
 * 0 switches every probe off. */
void pipck_tune_probes(uint32_t probes);

/* The ring verifier's schedule switches (pipck_rx_verify_ring; process-wide,
 * internal, every setting gives the same verdicts; 0 = automatic: k_ring, and
 * for slot strides from 4 KiB k_ring or the row stream k_ring_rx as the
 * feedback of the same ring's earlier launches says it is full): bit 0 =
 * k_ring's row stream never deals items round-robin to the block's waves,
 * bit 1 = always; bit 2 = no feedback (k_ring at every fill, the round-5
 * default); bit 3 = the feedback at every stride. */
void pipck_tune_ring(uint32_t mode);

/* XCD-weighted static deal for k_flat (ring 24, checksum; measurement arm,
 * VERDICT r03 item 7): the grid is cut into periods of 8 x period blocks and
 * in each XCD x (blocks b with b % 8 == x) keeps its first m[x] blocks; the kept
 * blocks take the tasks in dispatch order.  m = NULL or period = 0 switches it
 * off.  Same results; only the share of tasks per XCD changes. */
int pipck_tune_xcd_weights(const uint32_t* m, uint32_t period);

/* Per-task timeline for tools/task_trace.py: with tune flags bit 20 set, the
 * flat-stream (k_flat) and packed ragged (k_packed) kernels store one record
 * {u64 task, u64 t_start, u64 t_end, u64 XCC_ID << 32 | HW_ID} per wave task
 * (100 MHz s_memrealtime clock) into d_buf[task] for task < cap.  d_buf is
 * device memory; null switches recording off. */
int pipck_trace_tasks(void* d_buf, uint64_t cap);

/* The demangled name of the batch kernel the calling thread launched last --
 * the exact template instantiation, spelled as rocprofv3 names it (e.g.
 * "void pipck::k_flat<32, true, false, true, 4>(unsigned char const*, ...)").
 * bench.py attaches a PMC traffic file to a bench line only when the file was
 * measured on this kernel of this build.  PIPCK_EINVAL before any launch. */
int pipck_last_launch(char* buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* PIPCK_TESTING_H */
