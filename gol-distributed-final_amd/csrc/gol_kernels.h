// gol_kernels.h -- internal launcher interface of gol_kernels.hip (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef GOL_COUNT_SLOTS
#define GOL_COUNT_SLOTS 256
#endif

// Flags of a launch's device error word (ORed by the failing waves).
#define GOLK_ERR_SPIN 1u  // a pipeline wave gave up waiting for an LDS flag (protocol fault)
#define GOLK_ERR_IPC 2u   // an IPC rank gave up waiting for a neighbour's flag (gol_comm.h)

// Per-device error word for launches made without one (lazily allocated, zeroed).
uint32_t *golk_device_err_word(int device);
// Per-device CU slot masks of the band pipeline's role placement (indexed by XCC, SE, SH, CU).
#define GOL_CU_SLOT_WORDS 2048
uint32_t *golk_cu_slots(int device);
// Zero them again on `s` (after a faulted launch whose workgroups may not have freed their slots).
hipError_t golk_reset_cu_slots(int device, hipStream_t s);
// Paired-rank claim counters (one buffer per launch stream, gol_kernels.hip StripMap).
// golk_reset_claims: zero the buffer of stream s, ordered on s (after a faulted launch).
// golk_release_claims: free it (the caller has synchronised s; an engine destroying its streams).
// golk_own_stream: mark s as an engine's stream; golk_reset_claims_device (gol_dev_error, after a
// fault in a launcher call on a caller's stream) then leaves its buffer alone.
hipError_t golk_reset_claims(hipStream_t s);
void golk_release_claims(hipStream_t s);
void golk_own_stream(hipStream_t s);
hipError_t golk_reset_claims_device(int device);

int golk_auto_strip(int64_t rows, int64_t ngroups, int k);
// Standard layout: dw words per lane (1, 2 or 4), k in {1, 2, 4, 8} (and 16 for dw <= 2).
hipError_t golk_bits_step(const uint32_t *top, const uint32_t *mid, const uint32_t *bot, uint32_t *dst,
                          int64_t R, int64_t Wd, int64_t pitch, int64_t row0, int64_t rows, int k, int dw,
                          int strip, uint64_t *slots, hipStream_t s);
// Band layout (bit b of word w = cell b*Wd + w): dw words per lane (2 or 4), k in {1, 2, 4, 8},
// 16 for dw = 2, 12 for dw = 4 (the split pipeline); Wd % dw == 0, pitch % dw == 0, 4*dw-byte
// aligned rows.  err: error word of the launch (NULL = the device's default word).
#ifndef GOL_BAND_DEFAULT_DW
#define GOL_BAND_DEFAULT_DW 4
#endif
hipError_t golk_band_step(const uint32_t *top, const uint32_t *mid, const uint32_t *bot, uint32_t *dst, int64_t R,
                          int64_t Wd, int64_t pitch, int64_t row0, int64_t rows, int k, int dw, int strip,
                          uint64_t *slots, uint32_t *err, hipStream_t s);
int golk_band_useful_words(int k, int dw);
// Rounds of resident workgroups a step launch over `rows` rows makes (the band pipeline: 1 for
// its one-round rank-weighted launch; other kernels: 1e9, i.e. many); for the engine's choice of
// step plan.
double golk_step_rounds(bool band, int64_t rows, int64_t Wd, int64_t pitch, int k, int dw, int strip);
// Standard <-> band rows (Wd % 32 == 0), out of place.
hipError_t golk_band_convert(bool to_band, const uint32_t *src, uint32_t *dst, int64_t rows, int64_t Wd,
                             int64_t spitch, int64_t dpitch, hipStream_t s);
hipError_t golk_bytes_step(const uint8_t *world, int64_t H, int64_t W, int64_t stride, int64_t y0, int64_t y1,
                           uint8_t *out, int64_t out_stride, hipStream_t s);
hipError_t golk_bytes_blocked(const uint8_t *top, const uint8_t *mid, const uint8_t *bot, uint8_t *dst, int64_t R,
                              int64_t W, int64_t pitch, int64_t row0, int64_t rows, int k, int strip, uint64_t *slots,
                              uint32_t *err, hipStream_t s);
hipError_t golk_nonbinary(const uint8_t *bytes, int64_t rows, int64_t W, int64_t stride, uint32_t *flag, hipStream_t s);
hipError_t golk_random_fill(uint32_t *dst, int64_t rows, int64_t grow0, int64_t W, int64_t pitch, uint64_t seed,
                            hipStream_t s);
hipError_t golk_popcount(const uint32_t *src, int64_t rows, int64_t Wd, int64_t pitch, uint64_t *slots,
                         hipStream_t s);
// out[i] = sum of the GOL_COUNT_SLOTS slots of slot array i (arrays of GOL_COUNT_SLOTS*8 uint64);
// the slots are left zeroed.
hipError_t golk_slots_reduce(uint64_t *slots, int64_t n, uint64_t *out, hipStream_t s);
hipError_t golk_hash(const uint32_t *src, int64_t rows, int64_t grow0, int64_t Wd, int64_t pitch, uint64_t *slots,
                     hipStream_t s);
hipError_t golk_count_bytes(const uint8_t *src, int64_t rows, int64_t W, int64_t stride, uint64_t *slots,
                            hipStream_t s);
hipError_t golk_pack(const uint8_t *bytes, int64_t rows, int64_t W, int64_t stride, uint32_t *bits, int64_t pitch,
                     uint32_t *nonbinary, hipStream_t s);
hipError_t golk_unpack(const uint32_t *bits, int64_t rows, int64_t W, int64_t pitch, uint8_t *bytes, int64_t stride,
                       hipStream_t s);
// Per-row counts and the row-major (x, y) list of alive cells; with prev != NULL of the cells
// whose alive state differs between board and prev (same layout and pitch).  y0 is added to
// the listed y (global row of the first row).
hipError_t golk_row_counts(bool bits_mode, const void *board, const void *prev, int64_t rows, int64_t width_units,
                           int64_t pitch, int64_t *out, hipStream_t s);
hipError_t golk_alive_list(bool bits_mode, const void *board, const void *prev, int64_t rows, int64_t width_units,
                           int64_t pitch, const int64_t *offs, int32_t *xy, int64_t cap, int64_t y0, hipStream_t s);

// IPC transport (gol_comm.h): set *flag = value with release ordering at system scope after the
// stream's earlier work; wait (one wave on the stream) until every flags[i] (i < n <= 4, other
// processes' flag words mapped through IPC) has reached `want` (wrap-safe sequence compare),
// then acquire; after timeout_ticks of s_memrealtime (100 MHz) without it, OR GOLK_ERR_IPC into err.
#define GOLK_IPC_MAX_WAIT 4
hipError_t golk_ipc_signal(uint32_t *flag, uint32_t value, hipStream_t s);
hipError_t golk_ipc_wait(const uint32_t *const *flags, int n, uint32_t want, uint64_t timeout_ticks, uint32_t *err,
                         hipStream_t s);
