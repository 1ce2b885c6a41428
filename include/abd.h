/*
 * libabd -- MI355X (gfx950) poisoned-audio training hot path, C ABI.
 *
 * The reference (quantum-bitss/Audio-Backdoor-Attack) is pure Python; its drop-in
 * boundary is a set of Python call signatures.  Each entry point below replaces the
 * reference interface cited next to it; the Python host package
 * (audio-backdoor-attack_amd/) binds these with ctypes and re-exports the reference
 * names.
 *
 * Conventions
 *   - Plain pointers and sizes only; no torch types.  Device pointers are HBM
 *     buffers owned by the caller; the library allocates device memory only inside
 *     *_create() (constant tables), never inside a launch.
 *   - Every launch is asynchronous on the given stream (a hipStream_t passed as
 *     void*; NULL = the legacy default stream) and is hipGraph-capture safe.
 *   - Return value: 0 on success, a hipError_t value or ABD_E_* on failure;
 *     abd_last_error() returns a thread-local description.
 */
#ifndef ABD_H_
#define ABD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* abd_stream_t;

#define ABD_OK 0
#define ABD_E_INVALID 1001
#define ABD_E_UNSUPPORTED 1002
#define ABD_E_WORKSPACE 1003

const char* abd_last_error(void);
int abd_version(void);

/* ------------------------------------------------------------------ features
 * Replaces prepare_dataset.py:35-47  MFCC(waveform, sample_rate, n_mfcc, n_fft, hop_length)
 *      (torchaudio T.MFCC: HTK mel, reflect pad) and
 *      utils/daba_selection_tools.py:16-22  librosa_MFCC(waveform, sample_rate, n_mfcc)
 *      (librosa: Slaney mel+norm, constant pad, n_fft 2048 / hop 512).
 * Output layout is what the callers feed the model: (B, 1, T, n_mfcc) fp32,
 * i.e. MFCC(...).numpy().T[np.newaxis] stacked (prepare_dataset.py:65). */
enum { ABD_MEL_HTK = 0, ABD_MEL_SLANEY = 1 };
enum { ABD_PAD_REFLECT = 0, ABD_PAD_CONSTANT = 1 };

typedef struct abd_mfcc_plan abd_mfcc_plan;

int abd_mfcc_plan_create(int sample_rate, int n_fft, int hop_length, int n_mels, int n_mfcc,
                         int mel_kind, int pad_mode, float top_db, int64_t length,
                         abd_mfcc_plan** plan);
void abd_mfcc_plan_destroy(abd_mfcc_plan* plan);
int abd_mfcc_plan_frames(const abd_mfcc_plan* plan);
/* fft_size = M (== n_fft, or the Bluestein length for non-{2,3,5}-smooth n_fft). */
int abd_mfcc_plan_describe(const abd_mfcc_plan* plan, int* fft_size, int* bluestein,
                           int* n_passes, int* radices /* >= 16 ints */);
size_t abd_mfcc_workspace_bytes(const abd_mfcc_plan* plan, int64_t batch);

/* Trigger injection fused into the feature load / epilogue.
 *   ADD        x + trigger                      ultrasonic.py:75,96 (trigger from
 *                                               utils/ultra_trigger.py:92-111, length L)
 *   SNR_WINDOW x[p:p+Lt] += sqrt(|x|^2/|t|^2 * 10^(-snr/10)) * t      flowmur.py:77-85
 *   HALF_MIX   x/2 outside, (x+t)/2 inside [p, p+Lt)                  flowmur.py:101-106
 *   DEPLOY     s=10^(30/20)|t|/|x|: (s x + t)/(s+1) inside, s x/(s+1) outside
 *                                  utils/flowmur_generate_trigger.py:49-62
 *   DEPLOY_CLAMP  DEPLOY then clamp(-1, 1): the trigger-optimisation input
 *                                  utils/flowmur_generate_trigger.py:91-92
 *   patch      MFCC[t0:t1, c0:c1] = value on poisoned rows        utils/badnet_trigger.py:18-27
 * poison (uint8 per batch row) selects the rows that are injected (NULL = all);
 * position (int32 per batch row) is the window start for the windowed modes. */
enum { ABD_INJECT_NONE = 0, ABD_INJECT_ADD = 1, ABD_INJECT_SNR_WINDOW = 2,
       ABD_INJECT_HALF_MIX = 3, ABD_INJECT_DEPLOY = 4, ABD_INJECT_DEPLOY_CLAMP = 5 };

typedef struct abd_inject {
  int mode;
  const float* trigger;
  int64_t trigger_len;
  const uint8_t* poison;
  const int32_t* position;
  float snr_db;
  int patch;
  int patch_t0, patch_t1, patch_c0, patch_c1;
  float patch_value;
  /* ragged rows (utils/daba_selection_tools.py:70-76): frames[row] = 1 + len/hop of the
   * clip, zero-extended in its row; the top_db max sees only those frames and later
   * frames are set to frame_pad (-200 there).  NULL = every row has all T frames. */
  const int32_t* frames;
  float frame_pad;
  /* optional (round 5): the SNR / DEPLOY scale of every row of the wave TABLE, indexed by the
   * table row (rows[u]), as abd_inject_row_scales() writes it for a resident table whose rows and
   * trigger do not change (flowmur.py mixes the trigger into each clip once, offline).  NULL = the
   * call computes the scales of its batch itself (one extra launch per call). */
  const float* row_scale;
} abd_inject;

/* wave: row-major utterances (row_stride floats apart, plan length samples each) in
 * HBM.  rows (int32[batch], NULL = 0..batch-1) gathers the batch from the table.
 * out: (batch, 1, T, n_mfcc).  workspace: abd_mfcc_workspace_bytes(plan, batch). */
int abd_mfcc_f32(const abd_mfcc_plan* plan, const float* wave, int64_t row_stride,
                 const int32_t* rows, int64_t batch, const abd_inject* inj, float* out,
                 void* workspace, size_t workspace_bytes, abd_stream_t stream);

/* The injected waveform itself (batch, length): the reference's bd_*_wav arrays
 * (ultrasonic.py:75, flowmur.py:85/106). */
int abd_inject_waveform_f32(const float* wave, int64_t row_stride, int64_t length,
                            const int32_t* rows, int64_t batch, const abd_inject* inj,
                            float* out, void* workspace, size_t workspace_bytes,
                            abd_stream_t stream);
size_t abd_inject_workspace_bytes(int64_t batch);

/* The SNR_WINDOW / DEPLOY scale of each of n_rows table rows (flowmur.py:77-80,
 * flowmur_generate_trigger.py:50-52) into scales[n_rows]: every row as if poisoned (inj->poison is
 * ignored), rows 0..n_rows-1 of the table.  For abd_inject.row_scale. */
int abd_inject_row_scales(const float* wave, int64_t row_stride, int64_t length, int64_t n_rows,
                          const abd_inject* inj, float* scales, abd_stream_t stream);

/* FlowMur trigger optimisation, backward half (utils/flowmur_generate_trigger.py:89-104):
 * given dmfcc = d loss / d MFCC (batch, 1, T, n_mfcc) of
 *     MFCC(clamp(deploy(wave, trigger, position), -1, 1))          (inj->mode DEPLOY_CLAMP;
 *     DEPLOY skips the clamp), write d loss / d trigger (trigger_len floats) into dtrigger.
 * flags: ABD_BWD_ACCUMULATE adds to dtrigger; ABD_BWD_FORWARD_IN_WORKSPACE says the same
 * workspace just ran abd_mfcc_f32 on these inputs (its leading abd_mfcc_workspace_bytes()
 * hold the dB values, maxima and SNR scales), so the forward is not recomputed.
 * The gradient flows through the top_db clamp (ties split
 * like torch.maximum / amax), the dB log, the mel projection, |STFT|^2, the framing and
 * reflect padding, the clamp, the mix and the SNR scale s = 10^(30/20)|t|/|w|.
 * Needs a non-Bluestein specialised FFT plan (n_fft 2048 or 400; flowmur uses 2048) and
 * inj->poison == NULL.  workspace: abd_mfcc_deploy_backward_workspace_bytes(). */
size_t abd_mfcc_deploy_backward_workspace_bytes(const abd_mfcc_plan* plan, int64_t batch,
                                                int64_t trigger_len);
enum { ABD_BWD_ACCUMULATE = 1, ABD_BWD_FORWARD_IN_WORKSPACE = 2 };
int abd_mfcc_deploy_backward(const abd_mfcc_plan* plan, const float* wave, int64_t row_stride,
                             const int32_t* rows, int64_t batch, const abd_inject* inj,
                             const float* dmfcc, float* dtrigger, int flags,
                             void* workspace, size_t workspace_bytes, abd_stream_t stream);

/* DABA int16 path: pydub gain + overlay (utils/daba_selection_tools.py:24-39).
 * host/trig int16 (batch rows of host_len / trig_len); gain per row is the LINEAR factor
 * pydub applies, db_to_float(po_db - trig.dBFS) = 10 ** (dB / 20) evaluated in double by the
 * caller (so audioop.mul's floor sees the same product); out int16 (batch, host_len). */
int abd_pydub_overlay_i16(const int16_t* host, int64_t host_len, const int16_t* trig,
                          int64_t trig_len, const double* gain, int64_t batch,
                          int16_t* out, abd_stream_t stream);

/* DABA selection front end (utils/daba_selection_tools.py:24-39 + the soundfile.read that
 * follows the wav export, :70): hosts of their own lengths host_len[row] (NULL = length),
 * row-major with host_stride; trig rows trig_stride apart (0 = one trigger for every row).
 * Writes `length` samples per row: the overlay inside the host, 0 past its end, as int16
 * (out_i16) and/or as float v/32768 (out_f32); either may be NULL. */
int abd_pydub_overlay_ragged_i16(const int16_t* host, int64_t host_stride, const int32_t* host_len,
                                 const int16_t* trig, int64_t trig_stride, int64_t trig_len,
                                 const double* gain, int64_t batch, int64_t length,
                                 int16_t* out_i16, float* out_f32, abd_stream_t stream);

/* utils/daba_selection_tools.py:55-65,78-81  F.softmax(output) + calc_ent (log2 entropy,
 * double accumulation) per row of log-probs; probs (n, K) optional. */
int abd_softmax_entropy(const float* logprobs, int64_t n, int num_classes, float* probs,
                        double* entropy, abd_stream_t stream);
/* utils/daba_selection_tools.py:67-68  cross_entropy(a, y) per row pair (float32, nan_to_num). */
int abd_pair_cross_entropy(const float* probs_a, const float* probs_y, int64_t n, int num_classes,
                           float* out, abd_stream_t stream);

/* ------------------------------------------------------------------ resampling
 * Replaces prepare_dataset.py:60  torchaudio.functional.resample(waveform, orig_freq, new_freq)
 * (sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99 by default): 16 kHz Speech
 * Commands -> 44.1 kHz for the ultrasonic attack.  Output length ceil(new * L / orig) on the
 * gcd-reduced rates.  Supported: <= 448 output phases and <= 176 taps after the gcd
 * reduction (16000 -> 44100 is 441 phases x 174 taps). */
typedef struct abd_resample_plan abd_resample_plan;
int abd_resample_plan_create(int orig_freq, int new_freq, int lowpass_filter_width, double rolloff,
                             abd_resample_plan** plan);
void abd_resample_plan_destroy(abd_resample_plan* plan);
int64_t abd_resample_output_length(const abd_resample_plan* plan, int64_t length);
/* in: batch rows of `length` samples, in_stride apart; out: rows of output_length, out_stride apart */
int abd_resample_f32(const abd_resample_plan* plan, const float* in, int64_t in_stride, int64_t batch,
                     int64_t length, float* out, int64_t out_stride, abd_stream_t stream);

/* ------------------------------------------------------------------ JingleBack style boards
 * Replaces utils/styles_trigger.py:8-53  get_boards() / poison_style(wav, board, sr), the
 * pedalboard (JUCE dsp, float32) chains jingleback.py applies to the poisoned clips.  A board
 * is a chain of up to 8 effects, each run like pedalboard does (reset=True: zero state, snapped
 * smoothers per clip).  Parameters p[] per kind (pedalboard argument order):
 *   GAIN        p0 gain_db
 *   DISTORTION  p0 drive_db                                   (tanh waveshaper after the gain)
 *   LADDER      p0 mode (0 LPF12, 1 HPF12, 2 BPF12, 3 LPF24, 4 HPF24, 5 BPF24), p1 cutoff_hz,
 *               p2 resonance, p3 drive                        (at most one per board)
 *   PHASER      p0 rate_hz, p1 depth, p2 centre_frequency_hz, p3 feedback, p4 mix (one per board)
 *   CHORUS      p0 rate_hz, p1 depth, p2 centre_delay_ms, p3 feedback (must be 0), p4 mix
 *               (its delay line reads the chain's input history: only memoryless effects
 *               may precede it, see below)
 *   REVERB      p0 room_size, p1 damping, p2 wet_level, p3 dry_level, p4 width, p5 freeze_mode
 *               (juce::Reverb mono, JUCE_UNDENORMALISE as on x86 builds; one per board;
 *               its comb / allpass buffers live in the caller's workspace)
 *   PITCHSHIFT  p0 semitones                                  (first effect of the board, at most one)
 *               pedalboard.PitchShift is Rubber Band (R2: phase-vocoder stretch by r = 2^(st/12),
 *               then a resample by 1/r); no bit-level spec is public, so this is a phase vocoder of
 *               the same structure defined in oracle/effects.py (pitch_shift): parity unpinned.
 *   Effects between the board's start (after a PitchShift) and a Chorus must be memoryless (Gain,
 *   Distortion): the chorus delay line re-applies them to the history it reads. */
enum { ABD_FX_GAIN = 0, ABD_FX_DISTORTION = 1, ABD_FX_LADDER = 2, ABD_FX_PHASER = 3, ABD_FX_CHORUS = 4,
       ABD_FX_REVERB = 5, ABD_FX_PITCHSHIFT = 6 };
typedef struct abd_effect {
  int kind;
  float p[8];
} abd_effect;
typedef struct abd_style_board abd_style_board;
int abd_style_board_create(const abd_effect* fx, int n, int sample_rate, int64_t max_length,
                           abd_style_board** board);
void abd_style_board_destroy(abd_style_board* board);
/* bytes of workspace abd_style_board_apply needs for `batch` clips of up to max_length samples
 * (0 without a Reverb or a PitchShift) */
size_t abd_style_board_workspace_bytes(const abd_style_board* board, int64_t batch);
/* out[u] = board(in[rows ? rows[u] : u]) for `length` samples (<= max_length) */
int abd_style_board_apply(const abd_style_board* board, const float* in, int64_t in_stride,
                          const int32_t* rows, int64_t batch, int64_t length, float* out,
                          int64_t out_stride, void* workspace, size_t workspace_bytes,
                          abd_stream_t stream);

/* ------------------------------------------------------------------ smallcnn
 * Replaces utils/models.py:17-65 smallcnn(num_classes, linear_features) forward /
 * backward, utils/training_tools.py:52-85 train() inner step (CrossEntropyLoss on
 * the log-probs, Adam step, loss/accuracy/ASR bookkeeping) and :87-134 test().
 *
 * Parameters live in ONE flat fp32 buffer in torch parameter order
 * (conv1.w, conv1.b, bn1.w, bn1.b, conv2.w, conv2.b, bn2.w, bn2.b, conv3.w, conv3.b,
 *  bn3.w, bn3.b, fc1.w, fc1.b, fc2.w, fc2.b) -- torch-layout views are handed to the
 * nn.Module, so state_dict()/checkpoints are the reference's.  Gradients and the
 * two Adam moments use the same flat layout. */
typedef struct abd_cnn abd_cnn;

int abd_smallcnn_create(int H0, int W0, int num_classes, int max_batch, abd_cnn** net);
/* GEMM precision of the conv2/conv3 forward, data- and weight-gradient products.
 * ABD_PREC_F32_SPLIT (the default of a new handle, the bench and the drop-in smallcnn): fp32
 * operands split exactly into three bf16 planes (x = x0 + x1 + x2) and multiplied as the six
 * terms with i + j <= 2 on v_mfma_f32_32x32x16_bf16 with fp32 accumulation -- every term exact,
 * dropped terms <= ~2^-26 |a*b| (below one fp32 rounding), i.e. fp32-accurate GEMMs, parity-tested
 * at the same 1e-4 fp32 tolerance as ABD_PREC_F32.  ABD_PREC_F32 (opt-in): fp32 MFMA
 * (v_mfma_f32_32x32x2_f32), slower.  ABD_PREC_BF16 (BASELINE configs[2]/[4]: "bf16, conv-as-GEMM
 * on MFMA"): operands rounded to bf16, fp32 accumulation; BatchNorm, fc layers and the loss stay
 * fp32. */
enum { ABD_PREC_F32 = 0, ABD_PREC_BF16 = 1, ABD_PREC_F32_SPLIT = 2 };
int abd_smallcnn_set_precision(abd_cnn* net, int precision);
void abd_smallcnn_destroy(abd_cnn* net);
int64_t abd_smallcnn_param_count(const abd_cnn* net);
/* offsets (floats) of the 16 parameter tensors inside the flat buffer */
int abd_smallcnn_param_offsets(const abd_cnn* net, int64_t* offsets /* 17 */);
int abd_smallcnn_flat_features(const abd_cnn* net);
size_t abd_smallcnn_workspace_bytes(const abd_cnn* net, int64_t batch);
/* Byte offset of a named activation buffer inside the workspace (tests / debugging):
 * p1 r2 p2 r3 p3d d2 logp dz dp3 da dz3 dp2 dz2 dp1 coef bcoef mask1 mask2 rowinfo p1s dz2s xh3. */
int64_t abd_smallcnn_workspace_offset(const abd_cnn* net, int64_t batch, const char* name);
/* 1 when abd_smallcnn_train_step at this batch folds BN1 into conv2 (ABD_PREC_F32_SPLIT; a step
 * with SyncBN (abd_train_args.bn_sync set) never folds): the workspace's p1 then holds m, the
 * pool1-selected relu(conv1) value per window, and p1 = alpha * m + beta' with BN1's coefficients
 * (coef[0][c] = (mean, invstd, alpha, beta')); 0 otherwise. */
int abd_smallcnn_bn1_folded(const abd_cnn* net, int64_t batch);
/* Plane count of the conv2 plane mode of abd_smallcnn_train_step at this batch (no SyncBN): 3
 * (ABD_PREC_F32_SPLIT) or 1 (ABD_PREC_BF16) when the step keeps conv2's two activation operands as
 * exact bf16 planes -- the workspace's "p1s" (pool1 output m, [planes][B*H1*W1p*64] uint16, replacing
 * p1) and "dz2s" (BN2 backward output, [planes][B*H2*W2*64], replacing dz2), x = sum of the planes
 * exactly for 3 planes, rne(x) for 1 -- else 0 (p1 / dz2 hold fp32). */
int abd_smallcnn_conv2_planes(const abd_cnn* net, int64_t batch);

/* Device-side counters written by the train/eval launches (int64 / double):
 *   [0] sum of per-batch mean losses (double bits; train steps weight each by
 *       grad_scale)  [1] samples  [2] correct
 *   [3] poisoned samples  [4] poisoned & predicted==label  [5] batches     */
#define ABD_METRICS_WORDS 8

typedef struct abd_train_args {
  const float* x;            /* (B,1,H0,W0) MFCC input                        */
  const int64_t* labels;     /* (B)                                           */
  const int64_t* indicators; /* (B) poison indicator, NULL = none             */
  int64_t batch;
  float* params;             /* flat                                          */
  float* grads;              /* flat (written)                                */
  float* exp_avg;            /* flat Adam m                                   */
  float* exp_avg_sq;         /* flat Adam v                                   */
  float* running;            /* 6 BN buffers packed: rm1,rv1,rm2,rv2,rm3,rv3  */
  int64_t adam_step;         /* step index after increment (1-based)          */
  float lr, beta1, beta2, eps;
  int do_update;             /* 0: forward/backward only (grads), 1: + Adam   */
  const uint8_t* mask1_in;   /* optional dropout keep masks (B,flat),(B,128)  */
  const uint8_t* mask2_in;   /*   NULL -> generated from (seed, counter)      */
  uint64_t seed, counter;
  uint8_t* mask1_out;        /* optional: masks used (for tests)              */
  uint8_t* mask2_out;
  float* logprobs_out;       /* optional (B,K)                                */
  int64_t* metrics;          /* ABD_METRICS_WORDS accumulators (device)       */
  float grad_scale;          /* multiply loss gradient (DP: B_local/B_global);
                              * also weights metrics[0]'s batch-mean loss, so
                              * the ranks' words sum to the global batch mean
                              * (uneven last batch included).  batch >= 1:
                              * a 1-row batch is valid (BatchNorm2d counts
                              * N*H*W elements per channel)                  */
  int64_t* num_batches_tracked; /* optional int64[3] (bn1..bn3), += 1          */
  void* fc_grads_event;      /* optional hipEvent_t, recorded on the stream once
                              * the fc1/fc2 gradients (flat tail from offset
                              * abd_smallcnn_param_offsets()[12]) are final, so
                              * a DP caller can start their all-reduce while the
                              * conv backward is still running               */
  int64_t row_offset;        /* DP: global batch row of this rank's row 0.  The
                              * generated dropout masks hash the GLOBAL element
                              * index, so N ranks on slices of one global batch
                              * draw exactly the masks one process would.     */
  /* Synchronised BatchNorm (optional; NULL = per-rank statistics like DDP).  At each of the
   * 6 BatchNorm reductions of a step (forward bn1..bn3, then backward bn3..bn1) libabd writes
   * this rank's per-channel double sums into bn_sync_buf + point * ABD_BN_SYNC_STRIDE
   * (2*C+1 doubles: [sum_c | sum2_c | element count] forward, [sum dy_c | sum dy*xhat_c | count]
   * backward) and calls bn_sync(ctx, point, offset, n) from the launching thread; the callback
   * must enqueue an in-place SUM all-reduce of those n doubles on `stream` (torch.distributed
   * on the current stream does).  The statistics then use the global sums and counts: the
   * normalisation, running statistics and input gradients equal one process's on the global
   * batch; BN weight/bias gradients stay this rank's share (summed by the gradient all-reduce). */
  double* bn_sync_buf;       /* device, >= 6 * ABD_BN_SYNC_STRIDE doubles               */
  int (*bn_sync)(void* ctx, int point, int64_t offset, int64_t n);
  void* bn_sync_ctx;
} abd_train_args;
#define ABD_BN_SYNC_STRIDE 136

int abd_smallcnn_train_step(abd_cnn* net, const abd_train_args* a, void* workspace,
                            size_t workspace_bytes, abd_stream_t stream);

/* Split step for data parallelism: forward+backward (grads), then the caller
 * all-reduces grads/BN stats, then abd_smallcnn_apply(). */
int abd_smallcnn_apply(abd_cnn* net, const abd_train_args* a, void* workspace,
                       size_t workspace_bytes, abd_stream_t stream);

/* Autograd path (nn.Module forward/backward outside the fused train()):
 * forward keeps every activation in the workspace; backward consumes d(log-probs)
 * and must follow the forward on the same workspace.  train_mode selects batch
 * statistics + dropout (a->mask*, seed, counter, running updated) vs running stats. */
int abd_smallcnn_forward(abd_cnn* net, const abd_train_args* a, int train_mode, void* workspace,
                         size_t workspace_bytes, abd_stream_t stream);
int abd_smallcnn_backward(abd_cnn* net, const abd_train_args* a, const float* dlogprobs,
                          void* workspace, size_t workspace_bytes, abd_stream_t stream);

/* A batch of independent batch-1 train-mode forwards (utils/daba_selection_tools.py:68-87
 * runs the freshly built, untrained model -- nn.Module defaults to train() -- on one clip at
 * a time): BatchNorm normalises each utterance by its OWN statistics, dropout is active
 * (masks from mask*_in or from (seed, counter)), running statistics are left untouched (the
 * reference's selection model is discarded).  logprobs (batch, K).
 * workspace: abd_smallcnn_forward_per_utterance_workspace_bytes(). */
size_t abd_smallcnn_forward_per_utterance_workspace_bytes(const abd_cnn* net, int64_t batch);
int abd_smallcnn_forward_per_utterance(abd_cnn* net, const float* x, int64_t batch, const float* params,
                                       uint64_t seed, uint64_t counter, const uint8_t* mask1_in,
                                       const uint8_t* mask2_in, float* logprobs, void* workspace,
                                       size_t workspace_bytes, abd_stream_t stream);

/* eval forward (model.eval()): running BN statistics, no dropout.  Writes log-probs
 * and, if labels != NULL, accumulates loss/correct/ASR counters like test(). */
int abd_smallcnn_eval(abd_cnn* net, const float* x, int64_t batch, const float* params,
                      const float* running, const int64_t* labels,
                      const int64_t* indicators, float* logprobs, int64_t* metrics,
                      void* workspace, size_t workspace_bytes, abd_stream_t stream);

/* Frozen-model input gradient (utils/flowmur_generate_trigger.py:98-103: the benign model,
 * saved by EarlyStoppingModel right after clean_test() and therefore in eval mode, with
 * requires_grad off): eval forward (running BN statistics, no dropout), CrossEntropyLoss on
 * the log-probs scaled by loss_scale (mean over the batch), backward to the input x.
 * Writes log-probs (B,K), dx (B,1,H0,W0) and, if metrics != NULL, accumulates the loss /
 * accuracy counters.  workspace: abd_smallcnn_input_grad_workspace_bytes(). */
size_t abd_smallcnn_input_grad_workspace_bytes(const abd_cnn* net, int64_t batch);
int abd_smallcnn_input_grad(abd_cnn* net, const float* x, int64_t batch, const float* params,
                            const float* running, const int64_t* labels, float loss_scale,
                            float* logprobs, float* dx, int64_t* metrics, void* workspace,
                            size_t workspace_bytes, abd_stream_t stream);

/* torch.optim.Adam single-tensor step over a flat buffer (weight_decay 0). */
int abd_adam_f32(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                 int64_t n, int64_t step, float lr, float beta1, float beta2, float eps,
                 abd_stream_t stream);

/* ------------------------------------------------------------------ profiling
 * Per-phase HIP-event brackets around libabd launches (bench.py roofline).  Bit i of
 * phase_mask enables phase i (see csrc/prof.h: 0 stft_mel, 1 db_dct, 6 conv2 fwd,
 * 20 conv2 wgrad, 21 conv2 dgrad, ...).  stop() synchronises the recorded events and
 * returns the summed milliseconds and launch counts per phase. */
int abd_profile_start(unsigned long long phase_mask, int max_records);
/* The same, bracketing only every `every`-th launch of each enabled phase (1, 1 + every, ...):
 * each bracket costs the stream a serialising timestamp (~4-5 us of idle GPU on MI355X), so
 * bench.py samples the launches of its timed steps instead of bracketing all of them. */
int abd_profile_start_every(unsigned long long phase_mask, int max_records, int every);
/* Mark the start of a step (call once per step, before its launches).  Once called, sampling
 * is per STEP: every launch of an enabled phase inside steps 0, every, 2 every, ... is bracketed
 * (launch-count sampling aliases with a phase launched several times per step). */
int abd_profile_step(void);
int abd_profile_stop(double* total_ms, int* counts, int n_phases);

#ifdef __cplusplus
}
#endif
#endif /* ABD_H_ */
