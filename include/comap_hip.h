/*
 * comap_hip.h -- C ABI of the MI355X-native COMAP hot path (gfx950 HIP).
 *
 * Drop-in boundary.  Each entry point names the reference
 * interface it replaces (paths relative to comancpipeline/ in
 * SharperJBCA/COMAPreduce v0.9.1):
 *
 *   comap_medfilt_f64        Tools/median_filter/medfilt.pyx:26-33
 *                            (medianFilter.cpp:4-30, Mediator.h:9-197)
 *   comap_bin_values_f64     Tools/binFuncs.pyx:7-32  (binValues)
 *   comap_l1_vane            Analysis/VaneCalibration.py:67-82,143-198
 *   comap_l1_atmosphere      Analysis/Level1Averaging.py:197-246
 *   comap_l1_average         Analysis/Level1Averaging.py:592-708,792-872
 *                            + Analysis/GainSubtraction.py:17-209
 *   comap_l1_channel_bin     Analysis/Level1Averaging.py:249-321 (Level1Averaging)
 *   comap_destripe_*         MapMaking/Destriper.py:85-263,402-503
 *   comap_prep_*             MapMaking/COMAPData.py:72-117,205-236,247-427,471-577
 *                            (read_comap_data / get_tod / read_pixels)
 *
 * Conventions
 *   - Plain C types only; no C++ exceptions cross this boundary.
 *   - Every function returns 0 on success, a negative code on failure; the
 *     message is available from comap_last_error(ctx).
 *   - "host" arguments are caller-owned host arrays; "dev" arguments are
 *     device pointers (hipMalloc'd / torch CUDA tensors) on ctx's device.
 *   - Work is enqueued on the context's stream (comap_set_stream); functions
 *     taking device pointers do not synchronise the host unless stated.
 *   - One context per host thread / process; a context is not thread-safe.
 *   - Pixel indices: int64 on the host API, int32 on device; -1 = off-map.
 */
#ifndef COMAP_HIP_H
#define COMAP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct comap_ctx comap_ctx;
typedef struct comap_l1_plan comap_l1_plan;
typedef struct comap_destriper comap_destriper;

/* ------------------------------------------------------------ context */
int comap_ctx_create(int device, comap_ctx **out);
int comap_ctx_destroy(comap_ctx *ctx);
const char *comap_last_error(const comap_ctx *ctx);
/* hip stream (hipStream_t as void*); NULL = the legacy default stream */
int comap_set_stream(comap_ctx *ctx, void *stream);
int comap_synchronize(comap_ctx *ctx);
/* Library build tag, e.g. "comap_hip gfx950 <date>" */
const char *comap_version(void);
/* Page-locked host memory from a process-wide cache (8 size classes per octave; a
 * freed block is kept for the next request of its class, up to COMAP_PINNED_CACHE_MB
 * cached): result buffers of device -> host copies that a caller keeps (the
 * destriper's maps) without paying hipHostMalloc (~2.5 ms for a 4-band map set) per
 * solve.  0 or -2 (out of memory).  Free a block only when no copy into it is pending. */
int comap_host_alloc(size_t bytes, void **out);
void comap_host_free(void *p);
/* The library keeps freed device temporaries (median plans, destriper problems) and
 * page-locked blocks cached for reuse, outside torch's allocator, up to
 * COMAP_TMP_CACHE_MB (default 16384) of device memory per device.  comap_cache_trim
 * waits for the cached blocks' last uses and returns them all to the system (device
 * pool trimmed to 0); comap_cache_bytes reports the current device's cached and live
 * temporary bytes and the cached page-locked bytes (any pointer may be NULL). */
int comap_cache_trim(void);
int comap_cache_bytes(int64_t *device_cached, int64_t *device_live, int64_t *host_cached);

/* ------------------------------------------------------------ drop-ins (host arrays) */
/* In place, identical to medfilt.medfilt(x, w) for any double input: NaN-free
 * x with n >= w takes the order-statistics kernels (out[i] = median of
 * x'[i-w/2 .. i-w/2+w-1] with x'[j<w/2] = x[0], x'[j>=n] = x[n-1]; even w
 * averages the two middle values); x holding NaN (every comparison of the
 * reference's two-heap with NaN is false, so its result follows the insertion
 * history), or ceil(w/2) <= n < w, is replayed exactly through the two-heap on
 * the device (Mediator.h:36-99, one workgroup per series).  Requires
 * n >= ceil(w/2): below it medianFilter.cpp reads and writes outside the array. */
int comap_medfilt_f64(comap_ctx *ctx, double *x_host, int64_t n, int32_t w);
/* Batched sliding median of nseries host series x[offsets[s]..offsets[s+1]).
 * mode 0: medfilt semantics (as comap_medfilt_f64) for every output;
 * mode 1: out = medfilt([x[::-1], x, x[::-1]], w)[n:2n], the reflect-padded
 * high-pass filter of Level1Averaging.median_filter / COMAPData.median_filter
 * (Level1Averaging.py:696-700, COMAPData.py:72-81), without materialising
 * the pad.  Series holding NaN or shorter than w take the two-heap replay (as
 * comap_medfilt_f64); every series needs ceil(w/2) values (mode 0) or
 * 3n >= ceil(w/2) (mode 1).  out_host has offsets[nseries] values. */
int comap_medfilt_batch_f64(comap_ctx *ctx, const double *x_host, const int64_t *offsets_host,
                            int32_t nseries, int32_t w, int32_t mode, double *out_host);
/* image[p] += weights[i] (or += 1 when weights == NULL) for 0 <= p < npix
 * and (mask == NULL || mask[i] != 0).  Accumulates into image in place. */
int comap_bin_values_f64(comap_ctx *ctx, double *image_host, int64_t npix,
                         const int64_t *pixels_host, const double *weights_host,
                         const int64_t *mask_host, int64_t n);

/* ------------------------------------------------------------ L1 -> L2 */
/* Observation description (device pointers).  Units are (feed, scan) pairs
 * the reduction processes: units[4*u + {0,1,2,3}] = {feed index, scan index,
 * first sample, n samples}. */
typedef struct {
    int32_t n_feeds;           /* F: feeds in the cube                     */
    int32_t n_bands;           /* must be 4                                */
    int32_t n_channels;        /* must be 1024                             */
    int32_t n_scans;           /* S                                        */
    int64_t n_samples;         /* T                                        */
    const float *tod;          /* dev f32 [F][4][1024][T]                  */
    const double *el;          /* dev f64 [F][T] (pixel_el, degrees)       */
    int32_t n_units;           /* U                                        */
    const int32_t *units_host; /* host int32 [U][4]                        */
} comap_obs_desc;

int comap_l1_plan_create(comap_ctx *ctx, const comap_obs_desc *desc, comap_l1_plan **out);
int comap_l1_plan_destroy(comap_l1_plan *plan);

/* Vane event [vane_start, vane_start + vane_len): per (feed, band) hot/cold
 * sample offsets (relative to vane_start) in CSR form on the host:
 * hot_idx[hot_off[fb] .. hot_off[fb+1]), fb = feed*4 + band; an empty hot
 * or cold list leaves that (feed, band) at 0 (reference RuntimeError path).
 * Writes tsys/gain dev f64 [F][4][1024] for this event. */
int comap_l1_vane(comap_l1_plan *plan, int64_t vane_start, int64_t vane_len,
                  const int32_t *hot_idx_host, const int64_t *hot_off_host,
                  const int32_t *cold_idx_host, const int64_t *cold_off_host,
                  double t_hot, double *tsys_dev, double *gain_dev);

/* Enqueue pass A (the per-channel moments AtmosphereRemoval needs) without
 * waiting, so host work can overlap it; the next comap_l1_atmosphere uses it. */
int comap_l1_prefetch(comap_l1_plan *plan);
/* AtmosphereRemoval: writes fit_values dev f64 [S][F][4][2][1024]
 * (offset, slope per channel; NaN outside the fitted channel set, or when
 * fewer than 100 samples are finite in all fitted channels -- select_time).
 * const_el_units_host lists the units whose scan is constant-elevation
 * (features == 9 throughout): their fit is (per-channel nanmedian, 0).  Also
 * caches the per-channel noise moments the Level-2 averaging reuses. */
int comap_l1_atmosphere(comap_l1_plan *plan, const int32_t *const_el_units_host, int32_t n_const_el,
                        double *fit_values_dev);

/* Level1AveragingGainCorrection.average_tod for every unit.
 *   fit_values dev [S][F][4][2][1024], tsys0/gain0 dev [F][4][1024]
 *   (vane event 0), calibrator != 0 for calibrator sources (per-channel
 *   nanmedian instead of the fit, no gain subtraction).
 * NaN samples inside the units are replaced IN PLACE in the device cube by
 * their channel's scan nanmedian (fill_bad_data) before the reduction.
 * Outputs dev f64 [F][4][T]: tod (gain-subtracted residual), tod_original,
 * weights.  Samples no unit of the plan covers (scan gaps, a C3 shard's foreign
 * units) are set to 0 here, so the outputs may be allocated uninitialised. */
int comap_l1_average(comap_l1_plan *plan, const double *fit_values_dev,
                     const double *tsys0_dev, const double *gain0_dev, int32_t calibrator,
                     double *tod_out_dev, double *orig_out_dev, double *weights_out_dev);

/* Level1Averaging.average_tod (Analysis/Level1Averaging.py:292-321): generic
 * 1/Tsys^2-weighted frequency binning of the whole cube.  Per (feed, band) and
 * bin k of bin_size channels: x = f32(d / gain_c), avg = sum_c x w_c / wsum_k,
 * stddev = sqrt(sum_c f32(x*x) w_c / wsum_k - avg^2), channel sums in channel
 * order.  weights/gain dev f64 [F][4][1024] (weights = 1/Tsys^2 with the edge
 * mask applied by the caller), wsum dev f64 [F][4][1024/bin_size];
 * avg/stddev dev f64 [F][4][1024/bin_size][T]. */
int comap_l1_channel_bin(comap_l1_plan *plan, int32_t bin_size, const double *weights_dev,
                         const double *gain_dev, const double *wsum_dev, double *avg_dev, double *stddev_dev);

/* Debug/inspection: copies internal per-unit arrays (host f64):
 * what = 0: normalisation rms [U][4][1024]; 1: median-filtered band mean
 * [F][4][T]; 2: dG [F][T]; 3: regression x0,x1 [U][4][1024][2]; 4: band mean
 * [F][4][T]; 5: kappa [3][U][4][1024]; 6: per-band constants [U][4][16];
 * 7: alpha [U][4][1024]; 8: offsets/slopes [U][4][1024][2]; 9: per (unit,
 * band) channel-list length and median-band flag [U][4][2]. */
int comap_l1_debug_fetch(comap_l1_plan *plan, int32_t what, double *out_host, int64_t n);

/* Per-kernel timing with HIP events recorded on the launching stream around
 * every launch (enable = 2) or around the three streaming passes only (enable =
 * 1: moments, band sums, regress).  collect synchronises, returns per-kernel total ms and launch
 * counts (ids: 0 vane, 1 moments/pass A, 2 atmos fit, 3 coef B, 4 band sums/
 * pass B, 5 sliding median, 6 series sums, 7 regress/pass C, 8 gain weights,
 * 9 coef D, 10 legacy pass D, 11 scan weights, 12 unused, 13 finish) and resets. */
int comap_l1_profile(comap_l1_plan *plan, int32_t enable);
int comap_l1_profile_collect(comap_l1_plan *plan, double *ms_host, int64_t *counts_host, int32_t n);

/* ------------------------------------------------------------ Level-2 spike mask */
/* Statistics.Spikes.run_fit_spikes (Analysis/Statistics.py:63-105) on a
 * device Level-2 TOD f64 [n_rows][T] (rows = feed*4 + band), scans from
 * edges_host [n_scans][2]: per row rms = tod_auto_rms (non-zero samples),
 * per scan medfilt(w = medfilt_window) high-pass, |x| > threshold*rms,
 * runs dilated as fit_spikes does with `step`.  mask_dev uint8 [n_rows][T]
 * (0 outside the scans).  Synchronises. */
int comap_spikes(comap_ctx *ctx, const double *tod_dev, int32_t n_rows, int64_t n_samples,
                 const int64_t *edges_host, int32_t n_scans, int32_t medfilt_window, int32_t step,
                 double threshold, uint8_t *mask_dev);

/* ------------------------------------------------------------ Level-2 power spectra (FFT noise QA) */
/* Positive-frequency power spectra of every (row, scan) of a device Level-2
 * TOD f64 [n_rows][T] (rows = feed*4 + band), scans from edges_host
 * [n_scans][2]; replaces the per-series np.fft calls of
 *   mode 0: Level2FitPowerSpectrum.run (Analysis/Level2Data.py:275-278),
 *           |fft(x)|**2 / n;
 *   mode 1: NoiseStatistics.power_spectrum (Analysis/Statistics.py:155),
 *           |fft(x)**2|.
 * mask_dev (optional, uint8 [n_rows][T]): masked samples are first replaced
 * by np.interp over the unmasked samples of the scan (Statistics.py:216-221).
 * Scan k writes out_dev[out_offsets_host[k] + r*nk + (j-1)] for
 * j = 1 .. nk = (n-1)/2 (fftfreq(n) > 0), n = scan length.  Synchronises. */
int comap_power_spectra(comap_ctx *ctx, const double *tod_dev, int32_t n_rows, int64_t n_samples,
                        const int64_t *edges_host, int32_t n_scans, const uint8_t *mask_dev, int32_t mode,
                        const int64_t *out_offsets_host, double *out_dev);

/* ------------------------------------------------------------ synthetic input (bench) */
/* Fills a device-resident synthetic observation with the statistics of
 * tod f32 [F][4][1024][T], band_average f32 [F][4][T].
 * level/mult/hot dev f64 [F][T] are the per-sample sky level (K),
 * multiplicative gain drift and hot-load excess prepared by the host.
 * feed0: index of the first generated feed in the whole observation (a feed
 * shard of an observation gets the same samples as the full cube). */
int comap_synth_tod(comap_ctx *ctx, int32_t n_feeds, int32_t feed0, int64_t n_samples, uint64_t seed,
                    const double *level_dev, const double *mult_dev, const double *hot_dev,
                    float *tod_dev, float *band_average_dev);

/* ------------------------------------------------------------ destriper */
/* Destriper problem on one rank (MapMaking/Destriper.py:155-263): samples
 * [N] with int32 pixel, f64 tod and weights, N a multiple of offset_length (<= 256;
 * calibrators use 250), map of npix pixels.  A negative pixel p (-1 = off-map) is never
 * binned, and its sample's projection reads m[npix + p] -- numpy's wrap in the
 * reference's m[pointing] (Destriper.py:206-213).  Builds the constant offset<->pixel
 * sparse operator and the sample-level maps once. */
int comap_destripe_create(comap_ctx *ctx, const int32_t *pixels_dev, const double *tod_dev,
                          const double *weights_dev, int64_t n_samples, int32_t offset_length,
                          int64_t npix, comap_destriper **out);
/* n_bands (1, 2 or 4) sidebands on the same pointing solved as one batched
 * system (run_destriper.py:146-189 loops the bands over one pointing):
 * tod/weights dev f64 [n_bands][N] band-major; keep_dev (optional, uint8
 * [n_bands][N/L]): 0 marks an offset the band's data prep dropped (all its
 * weights are 0 in that band; its samples are then left out of the band's
 * hit map, COMAPData.py:550-568).  Every per-band vector of the functions below
 * is interleaved band-fastest: offsets [N/L][n_bands], maps [npix][n_bands];
 * each band's CG keeps its own scalars, stop test and iteration count.
 * comap_destripe_create is this with n_bands = 1.
 * Offset order: the problem processes its offsets in an internal (spatially
 * sorted) order; every offset vector the functions below take or return is in
 * that order, except the x of comap_destripe_solve, which is in the caller's
 * order.  comap_destripe_offsets_natural converts an internal vector.
 * Returns -3 when a pixel index is >= npix or < -npix (checked on the device by the
 * set-up's count pass; the reference raises IndexError there, binning or reading m). */
int comap_destripe_create_bands(comap_ctx *ctx, const int32_t *pixels_dev, const double *tod_dev,
                                const double *weights_dev, const uint8_t *keep_dev, int64_t n_samples,
                                int32_t offset_length, int64_t npix, int32_t n_bands, comap_destriper **out);
/* comap_destripe_create_bands with the offsets' internal processing order given by the
 * caller: okey_dev int32 [N/L] with keys in [0, okey_max), the offsets sorted by it
 * (stable).  okey_dev NULL: the first on-map pixel of each offset (okey_max unused). */
int comap_destripe_create_keyed(comap_ctx *ctx, const int32_t *pixels_dev, const double *tod_dev,
                                const double *weights_dev, const uint8_t *keep_dev, const int32_t *okey_dev,
                                int64_t okey_max, int64_t n_samples, int32_t offset_length, int64_t npix,
                                int32_t n_bands, comap_destriper **out);
int comap_destripe_destroy(comap_destriper *d);
int64_t comap_destripe_n_offsets(const comap_destriper *d);
int32_t comap_destripe_n_bands(const comap_destriper *d);
/* x_out [N/L][NB] (caller's offset order) from x_internal (internal order); x_out != x_internal */
int comap_destripe_offsets_natural(comap_destriper *d, const double *x_internal_dev, double *x_out_dev);
int comap_destripe_nnz(const comap_destriper *d, int64_t *nnz_offset_major, int64_t *nnz_pixel_major);
/* Bytes one sparse-operator entry holds: 4 + n_bands (count form: every offset's
 * non-zero weights per band are one value, so an entry keeps uint8 sample counts;
 * COMAP_DS_CF=0 disables it) or 4 + 8 n_bands (f64 weight sums). */
int32_t comap_destripe_entry_bytes(const comap_destriper *d);
/* Padded entries of the projection's sliced-ELLPACK row copy (COMAP_DS_SELL=1; chunks of
 * 64 offsets padded to their longest row), or -1 when the problem has none. */
int64_t comap_destripe_sell_entries(const comap_destriper *d);
/* Local (this rank) sample-level maps, summed in binValues order:
 * h = sum w, hits = sum 1, naive_num = sum w tod (any may be NULL). */
int comap_destripe_local_maps(comap_destriper *d, double *h_dev, double *hits_dev, double *naive_num_dev);
/* mode 0: num = W x  (bin_offset_map of F x, local partial numerator);
 * mode 1: num = naive_num - W x (numerator of the destriped map). */
int comap_destripe_bin(comap_destriper *d, const double *x_dev, int32_t mode, double *num_dev);
/* y = F^T W (z - m[p]) with m = num/h (num where h == 0), z = F x; when
 * x_dev == NULL, z = tod (the CG right-hand side b).  h_dev == NULL uses the
 * local weight map.  dot_dev (optional, needs x) receives y.x. */
int comap_destripe_project(comap_destriper *d, const double *x_dev, const double *num_dev,
                           const double *h_dev, double *y_dev, double *dot_dev);
/* dot_dev[b] = sum a b over the N/L offsets, per band (fixed-order reduction) */
int comap_destripe_dot(comap_destriper *d, const double *a_dev, const double *b_dev, double *dot_dev);
/* alpha = rr/pq; x += alpha p; r -= alpha q; rr_new = r.r (device scalars) */
int comap_destripe_cg_update(comap_destriper *d, const double *rr_dev, const double *pq_dev,
                             double *x_dev, double *r_dev, const double *p_dev, const double *q_dev,
                             double *rr_new_dev);
/* beta = rr_new/rr; p = r + beta p */
int comap_destripe_cg_direction(comap_destriper *d, const double *rr_new_dev, const double *rr_dev,
                                double *p_dev, const double *r_dev);
/* Multi-rank CG iteration (Destriper.py:85-152 with p == pb), split at the
 * three cross-rank sums the caller performs between the calls (NB = bands):
 *   dist_bin        num = W p (local numerator)          -> all-reduce num
 *   dist_project    q = F^T W (F p - m[p]), m = num/h;
 *                   pq = local q.p                        -> all-reduce pq
 *   dist_update     alpha = rr/pq; x += alpha p; r -= alpha q;
 *                   rr_new = local r.r                    -> all-reduce rr_new
 *   dist_direction  p = r + (rr_new/rr) p; rr = rr_new; per band: count the
 *                   iteration, stop when rr_new/rr0 is NaN or below threshold.
 * scal_dev f64 [4 NB + 1], k-major: rr0[NB], rr[NB], pq[NB], rr_new[NB],
 * threshold; flags_dev int32 [2 + 2 NB]: all bands stopped, iterations any band
 * ran, stopped[NB], iterations[NB].  A stopped band is left unchanged and every
 * kernel returns at once when flags[0] is set, so a batch of iterations can be
 * queued with one host check of flags per batch (NB = 1: rr0, rr, pq, rr_new,
 * threshold / stop, iterations). */
int comap_destripe_dist_bin(comap_destriper *d, const double *p_dev, double *num_dev, const int32_t *flags_dev);
int comap_destripe_dist_project(comap_destriper *d, const double *p_dev, const double *num_dev,
                                const double *h_dev, double *q_dev, double *scal_dev, const int32_t *flags_dev);
int comap_destripe_dist_update(comap_destriper *d, double *scal_dev, double *x_dev, double *r_dev,
                               const double *p_dev, const double *q_dev, const int32_t *flags_dev);
int comap_destripe_dist_direction(comap_destriper *d, double *scal_dev, double *p_dev, const double *r_dev,
                                  int32_t *flags_dev);
/* The same iteration with the block PARTIALS of p.q and r.r all-reduced instead of
 * their sums, so no final-sum launches: the native solve's 4 kernels per iteration.
 * pq_part_dev / rr_part_dev f64 [NB][comap_destripe_dist_parts()], zeroed by the
 * caller before the first iteration (a rank writes its own blocks' slots; every rank
 * re-sums all slots in one fixed order, so the scalars agree across ranks).  scal as
 * above, with rr_new[NB] initialised to rr0 (the current r.r):
 *   dist_project_parts   q = F^T W (F p - m[p]); p.q partials -> all-reduce pq_part
 *   dist_update_fused    pq = sum(pq_part); x, r; r.r partials -> all-reduce rr_part
 *   dist_direction_fused rr_new = sum(rr_part); p = r + (rr_new/rr) p; stop test */
int32_t comap_destripe_dist_parts(void);
int comap_destripe_dist_project_parts(comap_destriper *d, const double *p_dev, const double *num_dev,
                                      const double *h_dev, double *q_dev, double *pq_part_dev,
                                      const int32_t *flags_dev);
int comap_destripe_dist_update_fused(comap_destriper *d, double *scal_dev, const double *pq_part_dev, double *x_dev,
                                     double *r_dev, const double *p_dev, const double *q_dev, double *rr_part_dev,
                                     const int32_t *flags_dev);
int comap_destripe_dist_direction_fused(comap_destriper *d, double *scal_dev, const double *rr_part_dev,
                                        double *p_dev, const double *r_dev, int32_t *flags_dev);
/* out = num/h (num where h == 0); h_dev == NULL uses the local weight map */
int comap_destripe_div_map(comap_destriper *d, const double *num_dev, const double *h_dev, double *out_dev);
/* Whole single-rank destriper_iteration (no collectives) for every band: CG
 * (one matvec per iteration, Destriper.py:85-152) to threshold / niter, then
 * the final maps.  Iterations run as replayed hipGraph batches on the
 * problem's own stream with device-side stop flags (identical iterates and
 * count to a per-iteration loop, per band).  Writes offsets x [N/L][NB] and
 * map/naive/weight/hits [npix][NB] (any map pointer may be NULL);
 * iters_out[b] = iterations band b performed.  Synchronises. */
int comap_destripe_solve(comap_destriper *d, double threshold, int32_t niter, double *x_dev,
                         double *map_dev, double *naive_dev, double *weight_dev,
                         double *hits_dev, int32_t *iters_out);
/* Pixel ids onto an internal map layout (the 2-D tiled layout of DeviceDestriper's
 * map_shape): out[i] = lut[p] for 0 <= p < npix, lut[npix + p] - n_internal for
 * -npix <= p < 0 (an unbinned sample's id p reads m[npix + p]: the negative id that
 * reads the same pixel of the internal map), n_internal for any other id (the set-up's
 * range check then rejects it, as it would the original).  Device pointers; one pass,
 * no host sync (replaces Destriper.py's row-major m[pointing] indexing order only). */
/* comap_relabel_pixels for the tiled layout itself (T x T tiles, T a power of two, row-major
 * tile order, Morton order inside: destriper.tiled_layout), the ids computed instead of
 * looked up; n_internal = ceil(nx / T) ceil(ny / T) T^2. */
int comap_relabel_pixels_tiled(comap_ctx *ctx, const int32_t *pix_dev, int64_t n, int64_t nx, int64_t ny, int32_t T,
                               int32_t *out_dev);
/* Offset order keys for a row-major nx x ny map: key_dev[o] = lut[round(mean y) nx +
 * round(mean x)] over offset o's samples with 0 <= p < nx ny (the internal id of the
 * offset's centroid pixel), n_internal for an offset with none.  The offsets crossing a
 * pixel then sit near each other in the internal order (the CG bin's x gathers). */
int comap_offset_centroid_keys(comap_ctx *ctx, const int32_t *pix_dev, int64_t n, int32_t offset_length, int64_t nx,
                               int64_t ny, const int32_t *lut_dev, int64_t n_internal, int32_t *key_dev);
int comap_relabel_pixels(comap_ctx *ctx, const int32_t *pix_dev, int64_t n, const int32_t *lut_dev, int64_t npix,
                         int64_t n_internal, int32_t *out_dev);

/* ------------------------------------------------------------ destriper data prep (COMAPData.py) */
/* One Level-2 file's inputs to comap_prep_gather (device pointers).  Output row r
 * (0 <= r < n_rows = len(output_feed_index)) takes its tod / weights / az / el /
 * Sun coordinates from file feed row row_src[r] (-1: a bad feed, the row stays 0,
 * COMAPData.py:306-315) and its pointing from file feed row pix_src[r] (read_pixels'
 * row mapping, :423-424; -1: pixel 0).  Columns are the concatenated scans:
 * scans[s] = {first sample, N_s = floor((end - start) / L) L, first column}. */
typedef struct comap_prep_file {
    const double *tod;            /* [F][B][T] averaged_tod/tod or tod_original */
    int64_t tod_feed_stride, tod_band_stride;
    const double *az, *el, *ra, *dec;   /* [F][T] spectrometer/pixel_pointing/pixel_* */
    int64_t point_stride;
    const uint8_t *spike;         /* [F][B][T] spikes/spike_mask (0 / 1), or NULL */
    int64_t spike_feed_stride, spike_band_stride;
    int32_t n_rows, n_scans;      /* any n_scans >= 1 (up to 128 held in LDS, more searched in HBM) */
    int64_t datasize;             /* columns per output row */
    const int64_t *scans;         /* [n_scans][3] */
    const int32_t *row_src, *pix_src;   /* [n_rows] */
    const int64_t *row_feed;      /* [n_rows] feed id written to feedid */
    const double *row_cal;        /* [n_rows][4] calibration factor per output band */
    const double *row_w;          /* [n_rows][4] 1 / auto_rms^2 per output band */
    const double *row_pct;        /* [n_rows][4] az 10 / 90, el 10 / 90 percentiles */
    int32_t bands[4];             /* file band of output band k */
    int32_t n_bands;              /* 1..4 */
    double sun_rot[9];            /* healpy Rotator(rot=[sun ra, sun dec], inv=True) matrix */
    int64_t obsid;
    const int64_t *pixels;        /* [n_rows][datasize] precomputed pixel ids (HEALPix) or NULL */
} comap_prep_file;
/* CelestialWCS world -> pixel (CAR / SIN / TAN), transform_to_1d (COMAPData.py:83-117) */
typedef struct comap_prep_wcs {
    int32_t proj;                 /* 0 CAR, 1 SIN, 2 TAN */
    int32_t galactic;             /* 1: J2000 -> galactic first (gal_rot, COMAPData.py:411-415) */
    double eul[5];                /* wcslib celestial Euler angles: lng0, 90 - lat_p, phi_p, cos, sin */
    double crpix[2], cdelt[2];
    int64_t nx, ny;
    double gal_rot[9];
} comap_prep_wcs;
/* Flat outputs (read_comap_data's vectors); a file's block starts at `offset` */
typedef struct comap_prep_out {
    double *tod, *w;              /* [n_bands][band_stride] */
    int64_t band_stride;
    double *az, *el, *ra, *dec;   /* ra = Sun distance (deg), dec = Sun-centric colatitude (rad) */
    int64_t *feedid, *obsid;
    int32_t *pix;
    int64_t offset;
} comap_prep_out;
/* rms_dev[r] = COMAPData.auto_rms(x_r / scale[r]) (COMAPData.py:205-208), x_r =
 * x_dev + rows[r] * row_stride (n values): NumPy's nanstd, bit for bit. */
int comap_prep_auto_rms(comap_ctx *ctx, const double *x_dev, int64_t row_stride, const int32_t *rows_dev,
                        const double *scale_dev, int32_t nrows, int64_t n, double *rms_dev);
/* pct_dev[r] = np.percentile(az[good], (10, 90)), np.percentile(el[good], (10, 90)),
 * good = isfinite(az) (COMAPData.py:338-346), bit for bit. */
int comap_prep_percentiles(comap_ctx *ctx, const double *az_dev, const double *el_dev, int64_t row_stride,
                           const int32_t *rows_dev, int32_t nrows, int64_t n, double *pct_dev);
/* get_tod + read_pixels of one file into the flat outputs (COMAPData.py:247-427),
 * before the high-pass; `wcs` may be NULL when f->pixels is given. */
int comap_prep_gather(comap_ctx *ctx, const comap_prep_file *f, const comap_prep_wcs *wcs,
                      const comap_prep_out *out);
/* x[seg] -= median_filter(x[seg][keep], w) on keep = the non-zero samples of each
 * segment seg_dev[k] = {element offset, length} (COMAPData.py:72-81, 353-360; bad =
 * tod == 0, so NaN and +-inf stay in the median input as in the reference): segments of
 * <= 2w values take np.nanmedian, longer ones the running median -- the two-heap replay
 * for a segment holding NaN, whose result follows the reference's insertion history.
 * Synchronises (segment lengths size the median plan). */
int comap_prep_highpass(comap_ctx *ctx, double *x_dev, const int64_t *seg_dev, int32_t nseg, int32_t w);
/* NaN -> 0, keep[b][o] = any weight of offset o in band b non-zero, the union of kept
 * offsets compacted into `out` (COMAPData.py:550-568).  Synchronises; *n_kept_out =
 * kept offsets; keep_out_dev [n_bands][n_kept_cap]. */
int comap_prep_cut(comap_ctx *ctx, const comap_prep_out *in, int32_t n_bands, int64_t n_samples,
                   int32_t offset_length, const comap_prep_out *out, uint8_t *keep_out_dev,
                   int64_t n_kept_cap, int64_t *n_kept_out);

#ifdef __cplusplus
}
#endif
#endif /* COMAP_HIP_H */
