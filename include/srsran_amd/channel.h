/*
 * include/srsran_amd/channel.h -- time-domain channel emulators of the test generator, batched
 * over independent links on one GPU.  Each link is one instance of the reference's emulator object, with its own
 * seed / parameters and its own state carried from call to call, exactly as the reference's object keeps it:
 *
 *   mi355_channel_fading_*   srslte_channel_fading_t  (lib/src/phy/channel/fading.c:214-367, fading.h:38-78)
 *                            multipath Rayleigh fading (36.104 B.2 EPA / EVA / ETU + Doppler): per segment of at
 *                            most N/2 samples the Jakes tap gains at the segment's time, the taps' frequency
 *                            response, FFT -> multiply -> IFFT of the zero-padded segment and overlap-add with the
 *                            tail of the previous segment (path delay N/4 included, so inter-carrier interference
 *                            and the delay spread appear in the time domain)
 *   mi355_channel_delay_*    srslte_channel_delay_t   (lib/src/phy/channel/delay.c:26-133, delay.h:27-62)
 *                            sinusoidally varying integer delay through a FIFO
 *   mi355_channel_hst_*      srslte_channel_hst_t     (lib/src/phy/channel/hst.c:22-90, hst.h:28-55)
 *                            high-speed-train Doppler profile applied as a frequency shift per call
 *
 * Buffers are device pointers to interleaved complex float (cf_t) samples; in and out may alias only where the
 * reference allows it (fading: no; delay: no; hst: yes).  A call processes every link of the object; calls are
 * synchronous unless a stream is given.  Returns MI355_SUCCESS (0) or a negative MI355_ERROR_* code.
 */
#ifndef SRSRAN_AMD_CHANNEL_H
#define SRSRAN_AMD_CHANNEL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mi355_channel_fading mi355_channel_fading_t;

/* srslte_channel_fading_init (fading.c:214-296) for nlinks links: link i gets model ("epa5", "eva70", "etu300", ...;
 * "none" is rejected: its FFT size is undefined in the reference) at srate Hz and seeds[i] (std::mt19937 Jakes
 * phases).  max_nsamples bounds the samples of one execute call.  The FFT size N of the model is returned by
 * mi355_channel_fading_fft_size. */
int      mi355_channel_fading_create(mi355_channel_fading_t** q, int device, double srate, const char* model,
                                     const uint32_t* seeds, uint32_t nlinks, uint32_t max_nsamples);
uint32_t mi355_channel_fading_fft_size(const mi355_channel_fading_t* q);
/* srslte_channel_fading_execute (fading.c:334-367) on every link: in[i] -> out[i], nsamples each, starting at
 * init_time[i] seconds (host array); end_time[i] (may be NULL) receives the returned time. */
int  mi355_channel_fading_execute(mi355_channel_fading_t* q, const float* const* in, float* const* out, uint32_t nsamples,
                                  const double* init_time, double* end_time, void* stream);
void mi355_channel_fading_free(mi355_channel_fading_t* q);

/* srslte_timestamp_t (timestamp.h:40-43) */
typedef struct {
  int64_t full_secs;
  double  frac_secs;
} mi355_timestamp_t;

typedef struct mi355_channel_delay mi355_channel_delay_t;

/* srslte_channel_delay_init (delay.c:52-78) for nlinks links with the same profile. */
int  mi355_channel_delay_create(mi355_channel_delay_t** q, int device, float delay_min_us, float delay_max_us,
                                float period_s, float init_time_s, uint32_t srate_max_hz, uint32_t nlinks,
                                uint32_t max_len);
/* srslte_channel_delay_update_srate (delay.c:80-84): empties the FIFOs */
int  mi355_channel_delay_update_srate(mi355_channel_delay_t* q, uint32_t srate_hz);
/* srslte_channel_delay_execute (delay.c:95-133) on every link at timestamp ts[i] (host array); delay_nsamples[i]
 * (may be NULL) receives the delay applied. */
int  mi355_channel_delay_execute(mi355_channel_delay_t* q, const float* const* in, float* const* out, uint32_t len,
                                 const mi355_timestamp_t* ts, uint32_t* delay_nsamples, void* stream);
void mi355_channel_delay_free(mi355_channel_delay_t* q);

/* srslte_channel_hst_init + _update_srate (hst.c:24-45) and srslte_channel_hst_execute (hst.c:47-83) for nlinks
 * links with the same profile, link i at timestamp ts[i]; fs_hz[i] (may be NULL) receives the Doppler shift. */
int mi355_channel_hst_execute_batch(int device, float fd_hz, float period_s, float init_time_s, uint32_t srate_hz,
                                    const float* const* in, float* const* out, uint32_t len, uint32_t nlinks,
                                    const mi355_timestamp_t* ts, float* fs_hz, void* stream);

#ifdef __cplusplus
}
#endif

#endif
