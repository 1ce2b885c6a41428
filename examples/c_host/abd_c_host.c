/* A non-Python host of the libabd C ABI (include/abd.h): plain C, the HIP runtime for device
 * memory and a stream, no torch.  One batch of the ultrasonic hot path as the reference's
 * ultrasonic.py runs it (ultrasonic.py:73-86 trigger add + MFCC, utils/training_tools.py:52-85
 * train step, :87-134 eval forward):
 *
 *   abd_mfcc_f32 (ADD trigger on the poisoned rows) -> abd_smallcnn_eval -> abd_smallcnn_train_step
 *
 * Inputs are raw little-endian files written by the caller (tests/test_gpu_c_host.py):
 *   DIR/waves.f32 (B x L), DIR/trigger.f32 (L), DIR/poison.u8 (B), DIR/params.f32 (flat, torch
 *   parameter order), DIR/running.f32 (320), DIR/labels.i64 (B), DIR/ind.i64 (B)
 * Outputs, beside them:
 *   mfcc.f32 (B x T x C), logp_eval.f32 (B x K), logp_train.f32 (B x K), mask1.u8 (B x flat),
 *   mask2.u8 (B x 128), grads.f32, params_after.f32, running_after.f32, metrics.i64
 *   (ABD_METRICS_WORDS)
 *
 *   usage: abd_c_host DIR B K
 * Exit status 0 on success; every libabd / HIP failure prints its message and exits 1. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "abd.h"

#define L_SAMPLES 44100
#define N_MFCC 40

static void die(const char* what, const char* msg) {
  fprintf(stderr, "abd_c_host: %s: %s\n", what, msg);
  exit(1);
}
#define HIPCHK(x)                                         \
  do {                                                    \
    hipError_t e_ = (x);                                  \
    if (e_ != hipSuccess) die(#x, hipGetErrorString(e_)); \
  } while (0)
#define ABDCHK(x)                             \
  do {                                        \
    if ((x) != ABD_OK) die(#x, abd_last_error()); \
  } while (0)

static void* read_file(const char* dir, const char* name, size_t bytes) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "rb");
  if (!f) die("open", path);
  void* p = malloc(bytes ? bytes : 1);
  if (!p) die("out of host memory", path);
  if (fread(p, 1, bytes, f) != bytes) die("short read", path);
  fclose(f);
  return p;
}

static void write_file(const char* dir, const char* name, const void* p, size_t bytes) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "wb");
  if (!f || fwrite(p, 1, bytes, f) != bytes) die("write", path);
  fclose(f);
}

/* host buffer -> new device buffer */
static void* to_device(const void* h, size_t bytes) {
  void* d = NULL;
  HIPCHK(hipMalloc(&d, bytes ? bytes : 1));
  if (bytes) HIPCHK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
  return d;
}

static void to_file(const char* dir, const char* name, const void* d, size_t bytes) {
  void* h = malloc(bytes ? bytes : 1);
  if (!h) die("out of host memory", name);
  HIPCHK(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
  write_file(dir, name, h, bytes);
  free(h);
}

int main(int argc, char** argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: %s DIR B K\n", argv[0]);
    return 2;
  }
  const char* dir = argv[1];
  const int64_t B = atoll(argv[2]);
  const int K = atoi(argv[3]);
  if (B < 1 || B > (1 << 20) || K < 2) die("arguments", "B >= 1 and K >= 2 required (B <= 2^20)");
  hipStream_t stream;
  HIPCHK(hipStreamCreate(&stream));

  /* ---- features: ultrasonic.py's MFCC(wav + trigger, 44100, 40, 1103, 441) on the device */
  abd_mfcc_plan* plan = NULL;
  ABDCHK(abd_mfcc_plan_create(44100, 1103, 441, 128, N_MFCC, ABD_MEL_HTK, ABD_PAD_REFLECT, 80.0f, L_SAMPLES, &plan));
  const int T = abd_mfcc_plan_frames(plan);
  float* h_waves = read_file(dir, "waves.f32", (size_t)B * L_SAMPLES * sizeof(float));
  float* h_trig = read_file(dir, "trigger.f32", (size_t)L_SAMPLES * sizeof(float));
  uint8_t* h_pois = read_file(dir, "poison.u8", (size_t)B);
  float* d_waves = to_device(h_waves, (size_t)B * L_SAMPLES * sizeof(float));
  float* d_trig = to_device(h_trig, (size_t)L_SAMPLES * sizeof(float));
  uint8_t* d_pois = to_device(h_pois, (size_t)B);
  float* d_x = NULL;
  HIPCHK(hipMalloc((void**)&d_x, (size_t)B * T * N_MFCC * sizeof(float)));
  size_t ws_bytes = abd_mfcc_workspace_bytes(plan, B);
  void* d_ws = NULL;
  HIPCHK(hipMalloc(&d_ws, ws_bytes));
  abd_inject inj;
  memset(&inj, 0, sizeof inj);
  inj.mode = ABD_INJECT_ADD;
  inj.trigger = d_trig;
  inj.trigger_len = L_SAMPLES;
  inj.poison = d_pois;
  ABDCHK(abd_mfcc_f32(plan, d_waves, L_SAMPLES, NULL, B, &inj, d_x, d_ws, ws_bytes, stream));

  /* ---- smallcnn(K, 3072) on the (B, 1, T, 40) features */
  abd_cnn* net = NULL;
  ABDCHK(abd_smallcnn_create(T, N_MFCC, K, (int)B, &net));
  const int64_t np_ = abd_smallcnn_param_count(net);
  const int flat = abd_smallcnn_flat_features(net);
  float* h_params = read_file(dir, "params.f32", (size_t)np_ * sizeof(float));
  float* h_running = read_file(dir, "running.f32", 320 * sizeof(float));
  int64_t* h_labels = read_file(dir, "labels.i64", (size_t)B * sizeof(int64_t));
  int64_t* h_ind = read_file(dir, "ind.i64", (size_t)B * sizeof(int64_t));
  float* d_params = to_device(h_params, (size_t)np_ * sizeof(float));
  float* d_running = to_device(h_running, 320 * sizeof(float));
  int64_t* d_labels = to_device(h_labels, (size_t)B * sizeof(int64_t));
  int64_t* d_ind = to_device(h_ind, (size_t)B * sizeof(int64_t));
  float *d_grads = NULL, *d_m = NULL, *d_v = NULL, *d_lp = NULL, *d_lpt = NULL;
  uint8_t *d_m1 = NULL, *d_m2 = NULL;
  int64_t* d_metrics = NULL;
  HIPCHK(hipMalloc((void**)&d_grads, (size_t)np_ * sizeof(float)));
  HIPCHK(hipMalloc((void**)&d_m, (size_t)np_ * sizeof(float)));
  HIPCHK(hipMalloc((void**)&d_v, (size_t)np_ * sizeof(float)));
  HIPCHK(hipMemset(d_m, 0, (size_t)np_ * sizeof(float)));
  HIPCHK(hipMemset(d_v, 0, (size_t)np_ * sizeof(float)));
  HIPCHK(hipMalloc((void**)&d_lp, (size_t)B * K * sizeof(float)));
  HIPCHK(hipMalloc((void**)&d_lpt, (size_t)B * K * sizeof(float)));
  HIPCHK(hipMalloc((void**)&d_m1, (size_t)B * flat));
  HIPCHK(hipMalloc((void**)&d_m2, (size_t)B * 128));
  HIPCHK(hipMalloc((void**)&d_metrics, ABD_METRICS_WORDS * sizeof(int64_t)));
  HIPCHK(hipMemset(d_metrics, 0, ABD_METRICS_WORDS * sizeof(int64_t)));
  size_t cnn_ws_bytes = abd_smallcnn_workspace_bytes(net, B);
  void* d_cnn_ws = NULL;
  HIPCHK(hipMalloc(&d_cnn_ws, cnn_ws_bytes));

  /* test(): model.eval() forward with the running statistics (utils/training_tools.py:87-134) */
  ABDCHK(abd_smallcnn_eval(net, d_x, B, d_params, d_running, NULL, NULL, d_lp, NULL, d_cnn_ws, cnn_ws_bytes, stream));
  /* hipMemcpy below synchronises the default stream only: wait for ours first */
  HIPCHK(hipStreamSynchronize(stream));
  to_file(dir, "logp_eval.f32", d_lp, (size_t)B * K * sizeof(float));

  /* train(): zero_grad, forward (batch BN statistics, dropout), CE on log-probs, backward, Adam
   * (utils/training_tools.py:52-85 with Adam(lr=1e-4)); the dropout masks it draws are returned */
  abd_train_args a;
  memset(&a, 0, sizeof a);
  a.x = d_x;
  a.labels = d_labels;
  a.indicators = d_ind;
  a.batch = B;
  a.params = d_params;
  a.grads = d_grads;
  a.exp_avg = d_m;
  a.exp_avg_sq = d_v;
  a.running = d_running;
  a.adam_step = 1;
  a.lr = 1e-4f;
  a.beta1 = 0.9f;
  a.beta2 = 0.999f;
  a.eps = 1e-8f;
  a.do_update = 1;
  a.seed = 35;
  a.counter = 0;
  a.mask1_out = d_m1;
  a.mask2_out = d_m2;
  a.logprobs_out = d_lpt;
  a.metrics = d_metrics;
  a.grad_scale = 1.0f;
  ABDCHK(abd_smallcnn_train_step(net, &a, d_cnn_ws, cnn_ws_bytes, stream));
  HIPCHK(hipStreamSynchronize(stream));

  to_file(dir, "mfcc.f32", d_x, (size_t)B * T * N_MFCC * sizeof(float));
  to_file(dir, "logp_train.f32", d_lpt, (size_t)B * K * sizeof(float));
  to_file(dir, "mask1.u8", d_m1, (size_t)B * flat);
  to_file(dir, "mask2.u8", d_m2, (size_t)B * 128);
  to_file(dir, "grads.f32", d_grads, (size_t)np_ * sizeof(float));
  to_file(dir, "params_after.f32", d_params, (size_t)np_ * sizeof(float));
  to_file(dir, "running_after.f32", d_running, 320 * sizeof(float));
  to_file(dir, "metrics.i64", d_metrics, ABD_METRICS_WORDS * sizeof(int64_t));
  printf("abd_c_host ok: B %lld T %d K %d params %lld flat %d\n", (long long)B, T, K, (long long)np_, flat);

  abd_smallcnn_destroy(net);
  abd_mfcc_plan_destroy(plan);
  void* bufs[] = {d_waves, d_trig, d_pois, d_x, d_ws, d_params, d_running, d_labels, d_ind, d_grads, d_m, d_v,
                  d_lp, d_lpt, d_m1, d_m2, d_metrics, d_cnn_ws};
  for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; ++i) HIPCHK(hipFree(bufs[i]));
  HIPCHK(hipStreamDestroy(stream));
  free(h_waves);
  free(h_trig);
  free(h_pois);
  free(h_params);
  free(h_running);
  free(h_labels);
  free(h_ind);
  return 0;
}
