/* liblaspj A/B knobs (laspj_ctx_set_tuning): kernel variants and launch shapes that the
 * benchmarks sweep and the tests force, so every variant stays covered.  Not part of the
 * drop-in's contract — a NIF never sets them; every default (0) is the measured best on
 * MI355X (DESIGN.md §4 gives the measurements behind each). */
#ifndef LASPJ_TUNE_H
#define LASPJ_TUNE_H

#include "laspj.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LASPJ_TUNE_STREAM_GRID   1   /* workgroups for grid-stride streaming kernels    */
#define LASPJ_TUNE_STREAM_UNROLL 2   /* 16-B cells per lane per iteration: 1,2,4,8      */
#define LASPJ_TUNE_STREAM_NT     3   /* 1 = non-temporal loads/stores, 0 = default      */
#define LASPJ_TUNE_ETF_KERNEL    4   /* OR-Set payload writer: 0 = record kernel when the
                                        token images are uniform (24 KiB window; records
                                        staged per element when elements hold <= 8 token
                                        slots, spread over lanes otherwise), 1 = element
                                        staging, 2 / 3 = record kernel, lanes, 16 / 20 KiB,
                                        4 = record kernel, lanes, 24 KiB, 5 = record
                                        kernel, per element thread, 24 KiB.  0 also
                                        writes a NIF entry point's single merge in one
                                        launch with its join and size pass (look-back);
                                        any other value keeps them separate.  G-Set
                                        writer: few long payloads in chunks of 256 slots
                                        over the chip unless 6 (one wave per payload) or
                                        1 (one block per payload)                        */
#define LASPJ_TUNE_REDUCE_KERNEL 5   /* OR reduce over replica groups: 0 = tiles of 4
                                        cells per lane, one per block, when the replica
                                        length is a power of two and 2 <= group <= 4
                                        (4 = the same as a grid-stride sweep), 1 =
                                        per-replica segments with a
                                        compile-time group, 2 = generic segments (also
                                        the runtime-count loop of reduce_chunks);
                                        reduce_chunks at 2..8 chunks: tiles read one
                                        source at a time (stream unroll 2/4/8 cells per
                                        lane, default 4) unless 2, or 3 = grid-stride
                                        sweep with every chunk's load in flight       */
#define LASPJ_TUNE_PRODUCT_ROWS  6   /* rows per outer-product tile: 0 = default (256),
                                        32, 64, 128, 256                                */
#define LASPJ_TUNE_PRODUCT_COLS  7   /* columns per outer-product tile: 0 = default
                                        (1024), 2048, 4096                              */
#define LASPJ_TUNE_ETF_READ      8   /* OR-Set from_binary: 0 = batched records when the
                                        dictionary's record templates hash apart within
                                        every element, plus element batches when elements
                                        hold <= 8 token slots, and long payloads split
                                        between waves when there are few of them,
                                        1 = serial record scan, 2 = batched records
                                        without element batches, 3 = never split,
                                        4 = always split (256-byte segments),
                                        5 = always split (sized segments), 6 = element
                                        batches walked by the scalar unit (the lanes
                                        find element starts by default), 7 = no element
                                        batches for many-token dictionaries (one element
                                        at a time), 8 = the same as 0, 10 = as 0, with
                                        segment mode's redo pass as a launch of its own
                                        (by default the chain check's wave decodes a
                                        payload that failed it again itself).
                                        G-Set from_binary forms (the OR-Set decoders as
                                        with 0): 11 = round 4's (header by byte loads,
                                        a window per 256 elements, a payload's last 16
                                        bytes one element per window), 12 = 11 with the
                                        tail taken from the window, 13 = 4 elements per
                                        lane per round, 14 = 512-element chunks, 15 =
                                        the default form; 11..15 never take the split
                                        decoder of few long payloads (the default's
                                        element extents by one wave per payload, then
                                        the elements resolved over the chip)          */
#define LASPJ_TUNE_ETF_SEG       9   /* OR-Set from_binary segment bytes: 0 = sized by
                                        the launch (see LASPJ_TUNE_ETF_READ), else split
                                        every payload longer than this (>= 256, a
                                        multiple of 256)                               */
#define LASPJ_TUNE_LIST_WALK    10   /* list merges whose keys descend somewhere: 0 = the
                                        default (the chunked walk over the chip when an
                                        input is known not to ascend, else the one-wave
                                        run-jumping walk), 1 = one step per element,
                                        3 = the chunked walk whenever few replicas merge;
                                        2 = list_bind never takes its rank-indexed path
                                        (both lists ascending); for A/B               */
#define LASPJ_TUNE_NIF_PASSES   14   /* NIF entry points: device passes a call may take
                                        (0 = default 6; registering unseen terms, a grown
                                        answer area and a serial re-decode take one each).
                                        A call still unresolved after them answers
                                        LASPJ_NIF_FALLBACK — for tests of that guard      */
#define LASPJ_TUNE_LIST_CHUNK   15   /* rows per chunk of the list merges' chunked walk
                                        (0 = default: 1024, or more to keep <= 1024
                                        chunks; 64 .. 2^20)                             */
int         laspj_ctx_set_tuning(laspj_ctx* ctx, int knob, int64_t value);

#ifdef __cplusplus
}
#endif

#endif /* LASPJ_TUNE_H */
