/*
 * ouhip.h -- C ABI of the MI355X (gfx950) kernels behind open_universe_amd's
 * drop-in ``load_model()`` / ``model.enhance()`` surface.
 *
 * The reference (kolyangg/open-universe) is pure Python: its hot path is a
 * sequence of ATen ops issued from ``Universe.enhance``
 * (open_universe/networks/universe/universe.py:231-375) through the score and
 * conditioner networks.  Each entry point below replaces a run of those ops;
 * the reference interface it replaces is cited on each declaration.  The
 * Python host (open_universe_amd/_lib.py) binds these with ctypes.
 *
 * Conventions
 *  - All tensors are fp32 device pointers (caller-owned, hipMalloc'd or from
 *    the torch caching allocator); sizes are element counts; activations are
 *    NCW with the frame axis innermost (the reference's layout).
 *  - ``stream`` is a hipStream_t passed as void* (0 = null stream).
 *  - Every function returns 0 on success, a negative code on failure;
 *    ou_last_error() returns a thread-local message.  Nothing allocates device
 *    memory or synchronises, so every launch is hipGraph-capturable.
 */
#ifndef OUHIP_H
#define OUHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OUHIP_ABI_VERSION 8

int ou_abi_version(void);
const char* ou_last_error(void);

/* ------------------------------------------------------------------------
 * Fused implicit-GEMM 1-D convolution (kernels K1, K2, K3, K5, K8 of
 * SURVEY.md section 2.3).  Replaces PReLU_Conv.forward
 * (networks/universe/blocks.py:203-231) plus the ConvBlock arithmetic that
 * follows it (blocks.py:353-416: (h+res)/sqrt2, (cond_out+input_cond)/sqrt2,
 * film, conv stacks), the strided / transposed rate-change convolutions with
 * their binomial anti-alias FIRs folded into the weights (blocks.py:123-134,
 * 268-287), the 1x1 signal_cond_proj (score.py:166-171), the st_convs
 * (condition.py:33-65), the GRU input projection and the STFT-as-GEMM of the
 * mel front end (condition.py:85-108).
 *
 *   xv[c'][t] = prelu(in_scale[b] * x[b][c'%cin][t*R + c'/cin + shift])  (0 outside [0,in_len))
 *   (phase-major frame view: channel c' = ph*cin + ci; W's channel axis, as
 *   packed by ou_conv_pack, follows the same order)
 *   acc[m][u] = sum_{c',k} W[m][c'][k] * xv[c'][u + k - pad]     u in [f0, f0 + n_frames)
 *   m = ph*cout + co, t = u*rout + ph  (pixel shuffle; rout = 1 for plain convs)
 *   v = acc + bias[co];  v = t < valid_len ? v : 0
 *   v = (v + res1[b][co][t]) * s1;  v = film_g[b][co]*v + film_b[b][co];
 *   v = (v + res2[b][co][t]) * s2;  y[b][co][t] = v   for t < out_len
 * ---------------------------------------------------------------------- */
typedef struct ou_conv_desc {
    const float* x;            /* input signal                                   */
    int64_t x_bstride;         /* elements between batch items                   */
    int64_t x_cstride;         /* elements between channels                      */
    int32_t cin;               /* underlying input channels                      */
    int32_t in_len;            /* valid samples per channel                      */
    int32_t frame;             /* R: frame-view factor (1 = plain NCW)           */
    int32_t shift;             /* sample offset of frame 0                       */
    const float* in_scale;     /* [B] per-item input multiplier, or NULL         */
    float slope;               /* scalar PReLU slope (1.0 = identity)            */
    const float* w;            /* weights packed by ou_conv_pack()               */
    int32_t m;                 /* GEMM rows = rout * cout                        */
    int32_t kt;                /* taps along frames: 1, 3, 4 or 5                */
    int32_t pad;               /* left padding in frames                         */
    int32_t cc;                /* channel chunk the weights were packed with     */
    int32_t n_frames;          /* output frames u                                */
    int32_t batch;
    float* y;
    int64_t y_bstride, y_cstride;
    int32_t rout;              /* output phases (transposed conv), 1 otherwise;  */
                               /* < 0: |rout| phases with channel-major rows     */
                               /* m = co * |rout| + ph (else m = ph * cout + co) */
    int32_t out_len;           /* store t < out_len                              */
    int32_t valid_len;         /* t >= valid_len stored as 0 before res1         */
    const float* bias;         /* [cout] or NULL                                 */
    const float* res1;         /* residual 1 or NULL                             */
    int64_t r1_bstride, r1_cstride;
    float s1;
    const float* film;         /* [B][2*cout] (gamma | beta) or NULL             */
    int64_t film_bstride;
    const float* res2;         /* residual 2 or NULL                             */
    int64_t r2_bstride, r2_cstride;
    float s2;
    int32_t tile;              /* -1 = auto; bits 0-7 tile shape (< ou_conv_     */
                               /* num_tiles()), bits 8-9 log2(output tiles per   */
                               /* workgroup; > 0: persistent kernel, see         */
                               /* ou_conv_tile_ok)                               */
    int32_t prec;              /* 0: f32 operands (weights from ou_conv_pack);   */
                               /* 1: split-f16 operands (ou_conv_pack_split),    */
                               /*    f32-class accuracy, see ou_conv.hip;        */
                               /* 2: f16 operands (the hi halves of the same     */
                               /*    packing), f32 accumulation                  */
    float w_unscale;           /* prec 1: power of two from ou_conv_pack_split   */
    int32_t f0;                /* first output frame u computed: the launch      */
                               /* covers u in [f0, f0 + n_frames), in the global */
                               /* frame coordinates of x / y (zero padding only  */
                               /* at the true ends); 0 = from the start.  The    */
                               /* persistent / warp-specialised f32 kernels      */
                               /* (tile bits 8-10) need f0 = 0                   */
    int32_t* status;           /* prec 1 / 2: range codes (xs_shift) are OR-ed   */
                               /* in here, or NULL                               */
    float* ks_ws;              /* K-slice workspace (tile bits 12-13 = log2 S,   */
    int64_t ks_ws_bytes;       /* S > 1): S partial sums per output tile, then   */
                               /* a reduce + epilogue launch; NULL if unused     */
    /* Split images (prec 1).  The operand of the NEXT conv, stored once by
     * its producer's epilogue so that the consumer stages it with plain
     * copies: for every stored y[b][co][t] (rout 1)
     *   p = prelu_{sy_slope}(y) * 2^-sy_shift,  hi = f16(p),
     *   lo = f16((p - hi) * 2^11)
     * at byte (co / 32 * sy_rows + t) * 128 + (co % 32) * 2 (hi) and + 64
     * (lo) of item b: one 128-B row per 32-channel block and sample, the
     * channels of a block consecutive.  |p| >= 2^15 sets *status. */
    uint16_t* sy;              /* producer: also store y's split image, or NULL  */
                               /* (rout 1, m % 32 == 0, prec 1)                  */
    int64_t sy_bstride;        /* bytes between batch items                      */
    int32_t sy_rows;           /* samples per 32-channel block (>= out_len)      */
    int32_t sy_shift;          /* the consumer's staging exponent                */
    float sy_slope;            /* the consumer's PReLU slope                     */
    int32_t sy_pad_;
    const uint16_t* xs;        /* consumer (tile bit 15, conv_skernel): read the */
                               /* PReLU'd operand from this split image instead  */
                               /* of x (x, slope and in_scale unused; weights    */
                               /* from ou_conv_pack_split_nat; cin % 32 == 0)    */
    int64_t xs_bstride;        /* bytes between batch items                      */
    int32_t xs_rows;           /* samples per 32-channel block (>= in_len)       */
    int32_t xs_shift;          /* staging exponent s of every split-f16 / f16    */
                               /* kernel: the operand is staged (with xs: was    */
                               /* stored) as prelu(x) * 2^-s, |.| < 2^15.  A     */
                               /* larger staged value sets range code 1 in       */
                               /* *status, a larger split-image value (sy) 2, an */
                               /* infinite one 4; the engine then widens that    */
                               /* layer's exponent (default 6).  Bits 8 / 9 / 10 */
                               /* (with 1 / 2, ou_block's codes too): a finite   */
                               /* staged value reached 2^23 / 2^31 / 2^39        */
    /* Anti-aliased rate-change convs with the binomial FIR applied instead of
     * folded into the weights (tile bit 17; PReLU_Conv with use_antialiasing,
     * blocks.py:214-226, BinomialAntiAlias blocks.py:123-134):
     *   fir 1: f = FIR(prelu(x)) ('same', zero outside [0, in_len)), then the
     *          strided conv over f's frame view: frame = R, rout 1, K = cin R;
     *   fir 2: the transposed conv (frame 1, rout = -R, K = cin), then the FIR
     *          over its R * in_len output samples (zero outside), then bias.
     *   fir 3: no FIR: a plain strided conv (frame = R any multiple of 4,
     *          rout 1, K = cin R; the st_convs, condition.py:53-59) in fir 1's
     *          K order, walked so that each input sample is read once;
     * R is 2, 3, 4, 5 or 8 (fir 1 / 2); kt 1, pad 0, shift 0, no in_scale, no
     * xs; prec 1 or 2; weights w_logical[m'][k] packed by
     * ou_conv_pack_split_nat(kt 1):
     *   fir 1, 3: m' = co (m = cout rows), K in chunks of 16 channels x Q
     *          phases (Q = R for fir 1; 8 if R % 8 == 0 else 4 for fir 3),
     *          channel-major inside a chunk:
     *          k = ((cb R / Q + s) 16 + c) Q + p  for input channel
     *          ci = 16 cb + c (cin % 16 == 0) and conv tap ph = s Q + p
     *          (fir 1: k = ci R + ph, the frame view's order);
     *   fir 2: every 32-row m-tile holds P = 32 / R whole channels, row
     *          m' = 32 (co / P) + (co % P) R + ph (rows past P R zero), so
     *          ceil(cout / P) * 32 packed rows; k = ci (cin % 32 == 0).
     * fir 0: the other kernels (FIR folded into the weights). */
    int32_t fir;
    int32_t fir_pad_;
    const float* fir_taps;     /* [2R + 1] FIR taps (device; fir 1 / 2)          */
} ou_conv_desc;

/* Default channel chunk of the kernel for a tap count (informational: the
 * packed weight layout does not depend on it). */
int ou_conv_chunk(int kt, int frame);
/* Number of floats of the packed weight buffer. */
int64_t ou_conv_packed_size(int m, int cin_eff, int kt, int cc);
/* Host-side packing: w_logical[m][cin_eff][kt] (row-major, host memory)
 * -> packed[] in the per-lane MFMA fragment order the kernel streams:
 * [m-tile of 32][pair / 4][tap][lane][pair % 4], lane l holding row l & 31
 * and channel 2*pair + (l >> 5); channels padded with zeros to a multiple of
 * 64 (one float4 per lane = 4 consecutive k-steps of the MFMA stream). */
int ou_conv_pack(const float* w_logical, int m, int cin_eff, int kt, int cc,
                 float* packed);
/* Split-f16 packing (prec 1): the same number of floats as ou_conv_pack, in
 * the order [m-tile][8-pair group][hi | lo][tap][lane][8 halves] (lane l:
 * row l & 31, channel 2*(8*group + j) + (l >> 5) in half j) of
 * a = w * 2^e, hi = f16(a), lo = f16((a - hi) * 2^11), with e chosen per
 * layer so max|a| lies in [2^9, 2^10).  *w_unscale receives 2^(6-e) (the
 * kernel stages the input as x * 2^-6). */
int ou_conv_pack_split(const float* w_logical, int m, int cin_eff, int kt,
                       float* packed, float* w_unscale);
/* The same, in the natural channel order of the split-image kernel (tile bit
 * 15): [m-tile][16-channel group g][hi | lo][tap][lane][8 halves], lane l
 * holding row l & 31 and channel 16*g + 8*(l >> 5) + j in half j -- a lane's
 * B operand is then 8 consecutive channels of one split-image row. */
int ou_conv_pack_split_nat(const float* w_logical, int m, int cin_eff, int kt,
                           float* packed, float* w_unscale);
int ou_conv(const ou_conv_desc* d, void* stream);
/* The tile configuration ou_conv would use for this descriptor when
 * d->tile < 0; ou_conv_num_tiles() configurations exist, ou_conv_tile_ok()
 * says whether one fits the LDS budget for a tap count (host autotuning
 * times the valid ones per layer and stores the winner in d->tile). */
int ou_conv_pick_tile(const ou_conv_desc* d);
int ou_conv_num_tiles(void);
int ou_conv_tile_ok(int kt, int tile);
/* Diagnostics: LDS bytes a tile shape requests at tap count kt, and the
 * device's opt-in per-workgroup LDS limit. */
int ou_conv_lds_info(int kt, int tile, int* lds_request, int* device_optin_max);

/* ------------------------------------------------------------------------
 * Bidirectional GRU recurrence (kernel K6).  Replaces the recurrent part of
 * torch.nn.GRU in ScoreEncoder (score.py:84-90,117-118) and
 * ConditionerEncoder (condition.py:173-179,212-215).  The input projection
 * gi = W_ih x + b_ih is produced beforehand by ou_conv (1x1) into
 * gi[b][dir*3H + gate*H + j][t].  One persistent launch per layer: H/32
 * workgroups per direction hold W_hh in registers and hand h_t between
 * workgroups through 8-byte {tag, value} granules (bounded spins).
 *   y[b][dir*H + j][t] = (h + res[b][dir*H + j][t]) * res_scale   (res optional)
 * ---------------------------------------------------------------------- */
typedef struct ou_gru_desc {
    const float* gi;           /* [B][2*3H][T]                                    */
    int64_t gi_bstride;
    const float* w_hh;         /* [2][3H][H] (direction-major, torch layout)      */
    const float* b_hh;         /* [2][3H]                                         */
    float* y;                  /* [B][2H][T] (strides below)                      */
    int64_t y_bstride, y_cstride;
    const float* res;          /* optional residual, same layout as y             */
    int64_t res_bstride, res_cstride;
    float res_scale;
    int32_t hidden;            /* H: 256 or 384                                   */
    int32_t steps;             /* T                                               */
    int32_t batch;
    int32_t flags;             /* -1 default; bit0 XCD-local chains, bit1 spin    */
                               /* without s_sleep, bit2 64-unit workgroups, bit3  */
                               /* 128-unit workgroups, bit4 timing diagnostic     */
                               /* (skips the hand-off wait: wrong results), bit8  */
                               /* per-step gi prefetch instead of LDS-staged gi   */
                               /* chunks (one item per chain); bits 12-14 XCD     */
                               /* offset of the bit-0 chain layout, bit 15 keeps  */
                               /* the defaults of bits 0-11                       */
    uint64_t* granules;        /* workspace: ou_gru_workspace_bytes()             */
    int32_t* status;           /* device int, set nonzero on spin timeout         */
    int32_t t_begin, t_end;    /* steps [t_begin, t_end) of the T-step sequences  */
                               /* (forward: time t, backward: T - 1 - t); 0, 0 =  */
                               /* all.  A launch with t_begin > 0 starts from     */
                               /* hstate; every launch leaves h of its last step  */
                               /* there: the recurrence split over launches, each */
                               /* ordered after the one before (k-split kernel)   */
    float* hstate;             /* [B][2][H], or NULL (whole sequences only)       */
    int32_t ws_zeroed;         /* nonzero: the caller zeroed the workspace before */
                               /* the first launch on it (per replay); launches   */
                               /* leave it reusable, so no per-launch memset --   */
                               /* launches of steps < 5 clear it before and after */
                               /* they run (the tags T-1, T-2 a launch leaves     */
                               /* must not match a new launch's first two polls,  */
                               /* tags 1 and 2): launches of any T may share it   */
    int32_t _pad;
} ou_gru_desc;

int64_t ou_gru_workspace_bytes(int hidden, int batch);
int ou_gru(const ou_gru_desc* d, void* stream);

/* ------------------------------------------------------------------------
 * Noise-level embedding + every FiLM projection of the score network for a
 * list of sigma values (kernel K7).  Replaces SimpleTimeEmbedding /
 * SigmaBlock (sigma_block.py:24-78) and the per-level
 * Linear(noise_cond_dim -> 2C) calls (score.py:104-110,197-210).
 *   g = embed(log10(sigma[i]));  out[i][r] = sum_k W[r][k] g[k] + bias[r]
 * ---------------------------------------------------------------------- */
typedef struct ou_embed_desc {
    const float* sigma;        /* [n] noise levels (already scaled by edm.noise) */
    int32_t n;
    int32_t kind;              /* 0 = SimpleTimeEmbedding, 1 = SigmaBlock RFF    */
    int32_t dim;               /* noise_cond_dim (512)                           */
    float te_weight, te_bias;  /* SimpleTimeEmbedding scalars                    */
    const float* rff_freq;     /* SigmaBlock: [n_rff]                            */
    int32_t n_rff;
    int32_t rows;              /* total projection rows                          */
    const float* mlp_w[3];     /* SigmaBlock Linear weights (out x in)           */
    const float* mlp_b[3];
    float mlp_slope[3];
    const float* w;            /* [rows][dim] concatenated projections           */
    const float* bias;         /* [rows]                                         */
    float* out;                /* [n][rows]                                      */
    float* gbuf;               /* scratch [n][dim]                               */
} ou_embed_desc;

int ou_embed(const ou_embed_desc* d, void* stream);

/* ------------------------------------------------------------------------
 * Score-network head fused with the EDM wrapper and the sampler update
 * (kernel K9).  Replaces ScoreNetwork.forward's last two lines
 * (score.py:290-296: prelu -> output_conv), Universe._edm_score_wrapper
 * (universe.py:197-209) and the update lines of the diffusion loop
 * (universe.py:334-343).
 *   net = conv3(prelu2(prelu1(h)))[b][t] + bias
 *   mode 0: out = net
 *   else:   score = edm ? ((w_skip*x + w_out*net) - x) / s2 : net
 *   mode 1: out = (x + c_score*score) + c_noise*(z*s_next)
 *   mode 2: out = x + c_score*score
 * ---------------------------------------------------------------------- */
typedef struct ou_head_desc {
    const float* h;            /* [B][C][T] decoder output                       */
    int64_t h_bstride;
    int32_t channels, length, batch, mode;
    float slope1, slope2;
    const float* w;            /* [C][3] folded output_conv weight               */
    float bias;
    int32_t edm, _pad;
    float w_skip, w_out, s2, c_score, c_noise, s_next;
    const float* x;            /* [B][T] current sample (may alias out)          */
    const float* z;            /* [B][T] standard normal noise or NULL           */
    float* out;                /* [B][T]                                         */
} ou_head_desc;

int ou_head(const ou_head_desc* d, void* stream);

/* ------------------------------------------------------------------------
 * Row statistics and elementwise helpers around the sampler
 * (kernel K9): normalize_batch (utils/norm.py:47-87), the mel
 * normalization (condition.py:104-106), pad / unpad / peak-normalize /
 * keep_rms (universe.py:259,267-270,349-357).
 * ---------------------------------------------------------------------- */
/* y[b][i] = (x[b][i] - mean_b) * (level / max(std_b, eps)); std unbiased. */
int ou_normalize(const float* x, float* y, int batch, int64_t n, float level,
                 float eps, void* stream);
/* out[b] = 1 / max(sqrt(sum_i x[b][i]^2 / denom), eps)  (mel normalisation) */
int ou_inv_rms(const float* x, float* out, int batch, int64_t n, float denom,
               float eps, void* stream);
/* out[b] = sqrt(mean_i x[b][i]^2)                                          */
int ou_rms(const float* x, float* out, int batch, int64_t n, void* stream);
/* y[b][f][t] = x[b][f][t]^2 + x[b][f+F][t]^2   (|STFT|^2 from re/im rows)   */
int ou_power(const float* x, float* y, int batch, int nf, int frames, void* stream);
/* y[b][t] = x[b][t - left] for t-left in [0, n_in), 0 otherwise; len n_out  */
int ou_pad(const float* x, int64_t x_bstride, float* y, int batch, int n_in,
           int n_out, int left, void* stream);
/* y[i] = z[i] * scale (+ add[i])  (initial sample x0 = randn * sigma_0, or
 * the warm start aux + randn * sigma_k, universe.py:322-331)              */
int ou_scale(const float* z, float* y, int64_t n, float scale, const float* add,
             void* stream);
/* enhance() tail: crop [left, left+len) of x (stride x_bstride), optional
 * keep_rms rescale (mix_rms[b] / max(rms(x_b), 1e-5)), then divide by the
 * peak when it exceeds 1.                                                 */
int ou_finish(const float* x, int64_t x_bstride, int left, float* y, int batch,
              int len, const float* mix_rms, void* stream);
/* Elementwise median / mean over an ensemble of E results, [E][n] -> [n]
 * (universe.py:359-366: x.mean(dim=0) / x.median(dim=0).values, lower median). */
int ou_ensemble_reduce(const float* x, float* y, int ensemble, int64_t n,
                       int mode /* 0 mean, 1 median */, void* stream);
/* Ensemble signal_median (universe.py:366-367 -> utils/stats.py:22-66):
 * x [E][batch][n] -> y [batch][n] = the member selected by the reference's
 * per-sample rank vote.  counts: device int32 workspace [batch][32] (zeroed
 * here).  E <= 32. */
int ou_signal_median(const float* x, float* y, int ensemble, int batch, int64_t n, int* counts,
                     void* stream);

/* Audio-rate resampling around enhance(): replaces
 * torchaudio.functional.resample(x, orig, new) with its defaults
 * (sinc_interp_hann, lowpass width 6, rolloff 0.99) that the reference CLI
 * applies before and after the model (bin/enhance.py:61-64, 186-190).
 * orig/new reduced by their gcd; kernel = [phases = new][taps = 2*width + orig]
 * (dsp.sinc_resample_kernel); n_out = ceil(new * n_in / orig). */
int ou_resample(const float* x, int64_t x_bstride, float* y, int64_t y_bstride, int batch, int n_in,
                int n_out, const float* kernel, int phases, int taps, int orig, int width, void* stream);

/* FLAC input decoding for the CLI (host code): the
 * reference reads .wav/.mp3/.flac with torchaudio.load (bin/enhance.py:33,
 * 61-64); libFLAC / torchaudio are absent here.  ou_flac_info parses
 * STREAMINFO (frames = total samples per channel; counted by a decode pass
 * when STREAMINFO leaves it 0).  ou_flac_decode writes planar float32
 * out[c * frames + i] = sample / 2^(bps-1) (torchaudio.load's scaling) and
 * returns the frames decoded, or < 0 (ou_last_error) on a malformed stream or
 * a CRC-8 / CRC-16 mismatch. */
int ou_flac_info(const uint8_t* data, int64_t n, int32_t* sample_rate, int32_t* channels,
                 int32_t* bits_per_sample, int64_t* frames);
int64_t ou_flac_decode(const uint8_t* data, int64_t n, float* out, int64_t frames);
/* FLAC output (a .flac input is written back as .flac, as torchaudio.save
 * does): x planar float32 [channels][frames], PCM of bps = 16 or 24 bits
 * (round(x * 2^(bps-1)), clamped), FIXED-2 / VERBATIM subframes, CRCs set.
 * Returns the bytes written (<= ou_flac_encode_bound) or < 0. */
int64_t ou_flac_encode_bound(int channels, int64_t frames, int bps);
int64_t ou_flac_encode(const float* x, int channels, int64_t frames, int sample_rate, int bps, uint8_t* out,
                       int64_t capacity);

/* Alias-free Snake of the signal-decoupling layer (universe_gan.py:119-151;
 * bigvgan/snake.py:131-157, alias_free_act.py:8-30): torchaudio-style 2x
 * sinc up-sampling, Snake x + sin^2(a x)/(a + 1e-9), 2x down-sampling.  The
 * Conv1d(C -> 1, k3) that follows is ou_head in mode 0 with unit slopes.
 *   u[2s+i] = sum_k k_up[i][k] h[s+k-width_up];  y[t] = sum_k k_down[k] v[2t+k-width_down] */
typedef struct ou_snake_desc {
    const float* h;            /* [B][C][T]                                      */
    int64_t h_bstride;
    int32_t channels, length, batch, _pad0;
    const float* alpha;        /* [C] exp(log_alpha)                             */
    const float* k_up;         /* [2][taps_up]                                   */
    int32_t taps_up, width_up;
    const float* k_down;       /* [taps_down]                                    */
    int32_t taps_down, width_down;
    float* out;                /* [B][C][T]                                      */
} ou_snake_desc;

int ou_snake_aa(const ou_snake_desc* d, void* stream);

/* ------------------------------------------------------------------------
 * Fused ConvBlock main path (ou_block.hip): the three PReLU_Conv calls of a
 * ConvBlock and the arithmetic between them in one launch, for channel
 * counts whose whole channel range fits one workgroup (32, 64, 128, and
 * PP24's 48, 96 and 192; 256 and
 * 512 stay on ou_conv, see ou_block_supported) and
 * split-f16 / f16 / f32 operands.  Replaces blocks.py:393-416:
 *   c1 = conv1(h) (k5);  c1 = (c1 + sc) * s_sc;  c1 = film(c1);  cond_out = c1
 *   y  = ((h + conv3(conv2(c1))) * s_res + res2) * s2        (k3, k3)
 * Each conv applies its scalar PReLU slope to its input; frames outside
 * [0, length) are zero padding.  sc / film / cond_out / res2 are optional
 * (NULL).  y must not alias h, sc, cond_out or res2.
 * ---------------------------------------------------------------------- */
typedef struct ou_block_desc {
    const float* h;            /* block input [B][C][T]                          */
    int64_t h_bstride, h_cstride;
    int32_t channels, length;  /* C, T                                           */
    int32_t batch, prec;       /* prec 0 f32, 1 split-f16, 2 f16                 */
    const void* w[3];          /* conv1 (k5), conv2, conv3 (k3): ou_block_pack   */
    const float* bias[3];      /* [C] or NULL                                    */
    float slope[3];            /* PReLU slope on each conv's input               */
    float w_unscale[3];        /* from ou_block_pack                             */
    const float* sc;           /* conv1 residual (input_cond) or NULL            */
    int64_t sc_bstride, sc_cstride;
    float s_sc;
    int32_t dbg;               /* diagnostics only (tools/block_bench.py): 0     */
    const float* film;         /* [B][2C] (gamma | beta) or NULL                 */
    int64_t film_bstride;
    float* cond_out;           /* conv1 result after sc / FiLM, or NULL          */
    int64_t co_bstride, co_cstride;
    float* y;
    int64_t y_bstride, y_cstride;
    float s_res, s2;
    const float* res2;         /* or NULL                                        */
    int64_t r2_bstride, r2_cstride;
    int32_t* status;           /* split-f16 range flag (as ou_conv), or NULL     */
    /* 32 channels only, the score network's ends (both optional, NULL = off):
     * the block input is h = conv1d(in_scale[b] * x, w_in, b_in) (score
     * input_conv, 1 -> C, k3, score.py:244-246,285) instead of reading h;
     * and/or the block output goes through the score head (ou_head fields of
     * `head`; head.h is ignored) instead of being stored to y.            */
    const float* x;            /* [B][T] sampler state                           */
    int64_t x_bstride;
    const float* in_scale;     /* [B] or NULL                                    */
    const float* w_in;         /* [C][3]                                         */
    const float* b_in;         /* [C]                                            */
    ou_head_desc head;         /* head.w == NULL: no head                        */
    /* 32 / 64 channels (ou_block_down_supported): the encoder's strided
     * rate-change conv (blocks.py:203-231,268-275) on the block output, which
     * is still stored to y: e = conv(PReLU_down(y)) with stride `rate` and 2C
     * output rows over down_kt frames of `rate` samples per output frame
     * (down_kt 3: the anti-alias FIR folded in, frames -1, 0, +1; down_kt 1:
     * plain), zero outside [0, length).                                     */
    const void* w_down;        /* ou_block_pack_rect(2C, C, down_kt * rate) of
                                  the tap-major weights (tap k * rate + phase),
                                  or NULL: no rate-change conv                   */
    const float* b_down;       /* [2C] or NULL                                   */
    float slope_down, w_down_unscale;
    int32_t rate, down_kt;
    float* e;                  /* [B][2C][ceil(length / rate)]                   */
    int64_t e_bstride, e_cstride;
    /* Frame range (a chunk of a longer signal): outputs (y, cond_out, the
     * head, e) are computed and stored for frames [f0, f1) only, reading h
     * (x) wherever the convs' halos reach -- zero padding stays at [0,
     * length).  f1 = 0: the whole signal.  With a rate-change conv f0 and f1
     * are multiples of `rate`.  h frames outside [h0, h1) are read as zero
     * (h1 = 0: no limit): a chunk's caller has produced h only there, and
     * the frames it leaves out reach no stored output -- a workgroup past f1
     * stages them but stores nothing they feed.                             */
    int32_t f0, f1;
    int32_t h0, h1;
    /* Staging exponents (prec 1 / 2) of the conv1, conv2, conv3 and rate-
     * change conv inputs: each is staged as prelu(v) * 2^-shift (|.| < 2^15;
     * a larger value sets range code 1 / 2 / 8 / 16 in *status, an infinite
     * one 4).  The engine uses 6 unless a range flag widened a stage. */
    int32_t shift[4];
    /* Split images (prec 1; layout and values as ou_conv_desc.sy / xs).  sy:
     * also store the block output's image for the next conv (y is stored
     * too; not with a head; range code 32 when a value leaves the range).
     * xs: stage 0 copies the conv1 operand from this image (stored by the
     * producing conv with slope[0] and shift[0]) instead of staging h, which
     * is then read only as the residual (whole signal: f0 = f1 = h0 = h1 = 0,
     * no input conv). */
    uint16_t* sy;
    int64_t sy_bstride;        /* bytes between batch items                      */
    int32_t sy_rows, sy_shift; /* samples per 32-channel block; exponent        */
    float sy_slope;            /* the consumer's PReLU slope                     */
    int32_t sy_pad_;
    const uint16_t* xs;
    int64_t xs_bstride;        /* bytes between batch items                      */
    int32_t xs_rows, xs_pad_;  /* samples per 32-channel block (>= length)       */
} ou_block_desc;

/* 1 when ou_block handles this channel count and operand precision. */
int ou_block_supported(int channels, int prec);
/* Output frames per workgroup (the grid is ceil(length / frames) x batch). */
int ou_block_frames(int channels);
/* Halves of one packed conv (C x C x kt, hi and lo planes). */
int64_t ou_block_packed_halves(int channels, int kt);
/* Pack w[C][C][kt] (f32, host) as [m-tile][tap][16-channel step][hi | lo]
 * [lane][8 halves] of a = w * 2^e (max|a| in [2^9, 2^10)); *w_unscale =
 * 2^(6 - e). */
int ou_block_pack(const float* w, int channels, int kt, void* out, float* w_unscale);
/* The same packing for w[m][channels][kt] (m % 32 == 0, channels % 16 == 0):
 * the fused rate-change conv's 2C x C x (down_kt * rate) weights.            */
int ou_block_pack_rect(const float* w, int m, int channels, int kt, void* out, float* w_unscale);
/* f32 operands (prec 0): floats of the packed conv, and the packing
 * [m-tile][tap][4 channel pairs][lane][4] (lane l: row l & 31, channel
 * 2 pair + (l >> 5); rows padded to 32); *w_unscale = 2^6. */
int64_t ou_block_packed_f32(int channels, int kt);
int ou_block_pack_f32(const float* w, int channels, int kt, float* out, float* w_unscale);
/* 1 when ou_block fuses the rate-change conv for (channels, rate, kt, prec). */
int ou_block_down_supported(int channels, int rate, int kt, int prec);
int ou_block(const ou_block_desc* d, void* stream);

/* ------------------------------------------------------------------------
 * Program: a recorded list of the launches above, replayed natively (and
 * optionally as one hipGraph).  Built once per (shape, options) by the
 * Python host; replaces the Python-level loop of Universe.enhance.
 * ---------------------------------------------------------------------- */
typedef struct ou_program ou_program;

enum {
    OU_OP_CONV = 1, OU_OP_GRU = 2, OU_OP_EMBED = 3, OU_OP_HEAD = 4,
    OU_OP_NORMALIZE = 5, OU_OP_INV_RMS = 6, OU_OP_POWER = 7, OU_OP_PAD = 8,
    OU_OP_SCALE = 9, OU_OP_FINISH = 10, OU_OP_RMS = 11, OU_OP_SNAKE = 12,
    OU_OP_MEMSET = 13, OU_OP_ENSEMBLE = 14, OU_OP_BLOCK = 15,
    /* lanes: ops after OU_OP_LANE{id} run on stream `id` (0 = the caller's /
     * capture stream, id > 0 = program-owned side streams); OU_OP_SIGNAL{id}
     * records event id on the current lane, OU_OP_WAIT{id} makes the current
     * lane wait for it.  A side lane must start with a WAIT and lane 0 must end
     * after waiting for every side lane's last SIGNAL (checked: run and
     * capture fail otherwise).  ou_program_profile runs the list serially. */
    OU_OP_LANE = 16, OU_OP_SIGNAL = 17, OU_OP_WAIT = 18
};

/* Descriptors of the helper ops when recorded into a program. */
typedef struct ou_memset_desc {
    void* ptr;
    int64_t bytes;
} ou_memset_desc;
typedef struct ou_norm_args {
    const float* x;
    float* y;
    int32_t batch, _pad;
    int64_t n;
    float level, eps;
} ou_norm_args;
typedef struct ou_rms_args {
    const float* x;
    float* out;
    int32_t batch, _pad;
    int64_t n;
    float denom, eps;
} ou_rms_args;
typedef struct ou_power_args {
    const float* x;
    float* y;
    int32_t batch, nf, frames, _pad;
} ou_power_args;
typedef struct ou_pad_args {
    const float* x;
    int64_t x_bstride;
    float* y;
    int32_t batch, n_in, n_out, left;
} ou_pad_args;
typedef struct ou_scale_args {
    const float* z;
    float* y;
    int64_t n;
    float scale, _pad;
    const float* add;
} ou_scale_args;
typedef struct ou_finish_args {
    const float* x;
    int64_t x_bstride;
    int32_t left, batch, len, _pad;
    float* y;
    const float* mix_rms;
} ou_finish_args;
typedef struct ou_sync_args {
    int32_t id;                /* lane 0..8 (OU_OP_LANE) or event 0..4095 */
    int32_t _pad;
} ou_sync_args;
typedef struct ou_ensemble_args {
    const float* x;
    float* y;
    int32_t ensemble, mode;    /* mode 0 mean, 1 median, 2 signal_median   */
    int64_t n;                 /* batch * samples                          */
    int32_t batch, _pad;       /* signal_median: batch items (n / batch each) */
    int32_t* counts;           /* signal_median: [batch][32] int32 workspace */
} ou_ensemble_args;

ou_program* ou_program_create(void);
void ou_program_destroy(ou_program* p);
/* op-specific descriptor, copied into the program. */
int ou_program_add(ou_program* p, int op, const void* desc, size_t desc_bytes);
/* Replace the descriptor of op `index` (same kind and size; drops a captured
 * graph).  The recorder uses it to give a conv's epilogue a split-image
 * output (ou_conv_desc.sy) once it sees the conv that consumes it. */
int ou_program_patch(ou_program* p, int index, int op, const void* desc, size_t desc_bytes);
int ou_program_size(const ou_program* p);
int ou_program_run(ou_program* p, void* stream);
/* Capture the program into a hipGraph (on a private stream) and instantiate. */
int ou_program_capture(ou_program* p);
/* Host-only check of the lane structure (what run / capture validate
 * first): 0, or < 0 with ou_last_error.  No HIP call.                      */
int ou_program_validate(const ou_program* p);
/* Capture every maximal run of kernels on one lane (between two sync ops)
 * as its own hipGraph instead; ou_program_launch then replays the lanes on
 * real streams with host-side events, one graph launch per run.            */
int ou_program_capture_segments(ou_program* p);
/* Launch the captured program (whole graph, or segments) on ``stream``. */
int ou_program_launch(ou_program* p, void* stream);
/* Kind (OU_OP_*) of op i. */
int ou_program_op_kind(const ou_program* p, int i);
/* Eager replay with a hipEvent pair around every op on ``stream``; writes the
 * per-op device time in milliseconds to ms[0..size) (synchronises).  Used by
 * bench.py to attribute time to kernels inside the same workload. */
int ou_program_profile(ou_program* p, void* stream, float* ms);
/* Eager replay with the lanes on their streams (as ou_program_run) and a
 * hipEvent before and after every op on its lane: t0[i] / t1[i] = ms from the
 * replay's start to when op i's lane reached / finished it, -1 for sync ops
 * (synchronises).  The concurrent timeline of the lane schedule
 * (tools/critical_path.py). */
int ou_program_trace(ou_program* p, void* stream, float* t0, float* t1);

#ifdef __cplusplus
}
#endif
#endif /* OUHIP_H */
