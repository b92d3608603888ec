// Internals of librfx shared between its translation units (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rfx.h"

int rfx_detail_fail(int code, const char *msg);
uint32_t *rfx_detail_seed_word(rfx_renderer *r);  // device word holding the sphere stream's current state
uint32_t rfx_detail_jitter(const rfx_renderer *r);
void rfx_detail_set_jitter(rfx_renderer *r, uint32_t jitter);
hipStream_t rfx_detail_stream(const rfx_renderer *r);
void rfx_detail_set_rewindable(rfx_renderer *r, uint32_t jitter0);
// a frame of several passes: its start state saved on `st` before the first, then rewindable to it (rfx_frame_rng_rewind)
int rfx_detail_save_start(rfx_renderer *r, hipStream_t st);
void rfx_detail_set_rewindable_saved(rfx_renderer *r, uint32_t jitter0, hipStream_t st);
uint64_t rfx_detail_launch_traces(const rfx_renderer *r);
uint64_t rfx_detail_state_seq(const rfx_renderer *r);  // moves whenever the random streams move or are set
