/*
 * picotls/mi355x_debug.h -- test and measurement hooks of libptls_mi355x.so. Not part of the picotls drop-in boundary
 * (include/picotls/mi355x.h is); no reference counterpart. Used by tests/ and bench.py only.
 */
#ifndef picotls_mi355x_debug_h
#define picotls_mi355x_debug_h

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/**
 * Counters since the last reset, into out[16]:
 *   out[0..4]  launches of the chunked batch kernel per instantiation: 0 plain (4-bit GHASH tables), 1 spread (small
 *              batch with long records), 2 seal with header-protection masks, 3 W8 butterfly end (long whole records
 *              of a W8 pair), 4 W8 serial end (every other run of a W8 pair)
 *   out[5]     launches of the lockstep kernel, out[6] of the span kernels (a lone long record), out[7] 0
 *   out[8..12] runs processed on the device by each chunked instantiation (same order; a run skipped because the
 *              pair's other kernel takes it is not counted), out[13] 0, out[14] the EXT 4 runs among them that were
 *              multi-key runs (round 6: several connections' short records in one run), out[15] the EXT 4 runs
 *              processed in 4-lane groups (whole runs of short records of one key)
 * Waits for the whole device (reading the device counters). reset != 0 zeroes them after reading. Returns 0 or -1.
 */
int ptls_mi355x_debug_counters(uint64_t *out, int reset);

/**
 * Leaves a HIP error (hipErrorInvalidValue from hipHostGetDevicePointer on pageable memory) as the calling thread's last
 * error without clearing it, the state a handled failure used to leave behind. Returns the error code
 * left (0 if the call unexpectedly succeeded). The engine's calls on this thread must not be affected by it.
 */
int ptls_mi355x_debug_inject_error(void);

/**
 * Launches one wave on `stream` (a hipStream_t) that measures the shader clock of the CU it runs on over ~20 us: writes
 * three 64-bit words to the device-accessible `out`: shader-clock cycles (s_memtime) and real-time counter ticks
 * (s_memrealtime, rate ptls_mi355x_debug_wallclock_khz) elapsed over the same spin, and the XCD it ran on. Launched right
 * after a timed leg's last kernel, on its stream, it reads the clock the chip held under that load. Returns 0 or -1.
 */
int ptls_mi355x_debug_clock_sample(void *out, void *stream);
/* the real-time counter's rate in kHz (hipDeviceAttributeWallClockRate of the current device), 0 if unknown */
int ptls_mi355x_debug_wallclock_khz(void);

/**
 * Samples the shader clock inside the chunked batch kernels: from the next launch on, workgroup 0 of every chunked launch
 * that has work appends four 64-bit words to the device buffer `buf` (room for `cap` launches): shader-clock cycles
 * (s_memtime) at its start and end, then real-time counter ticks (s_memrealtime) at its start and end. buf = NULL stops
 * sampling. Waits for the device. Returns 0 or -1.
 */
int ptls_mi355x_debug_kernel_clock(void *buf, unsigned cap);
/* the number of launches sampled since the last ptls_mi355x_debug_kernel_clock (may exceed cap); waits for the device */
int ptls_mi355x_debug_kernel_clock_count(void);

#ifdef __cplusplus
}
#endif

#endif
