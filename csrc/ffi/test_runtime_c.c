/* C host program for the legacy FFModel runtime API (flexflow_runtime_c.h),
 * written the way the reference's Python package drove python/flexflow_c.h:
 * config -> model -> layers -> optimizer -> compile -> data loaders ->
 * epochs of forward / zero_gradients / backward / update -> metrics.
 * Exit status 0 = every check passed; prints one line per check. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "flexflow_runtime_c.h"

static int failures = 0;
#define CHECK(cond, ...)                 \
  do {                                   \
    if (cond) {                          \
      printf("ok   ");                   \
    } else {                             \
      printf("FAIL ");                   \
      ++failures;                        \
    }                                    \
    printf(__VA_ARGS__);                 \
    printf("\n");                        \
  } while (0)

enum { B = 32, F = 20, CLASSES = 4, SAMPLES = 256 };

/* synthetic, learnable: the label is the argmax of the first CLASSES features */
static void make_data(float* x, int* y) {
  unsigned s = 12345u;
  for (int i = 0; i < SAMPLES; ++i) {
    int best = 0;
    for (int j = 0; j < F; ++j) {
      s = s * 1103515245u + 12345u;
      x[i * F + j] = ((float)((s >> 8) & 0xffff) / 65535.f) * 2.f - 1.f;
      if (j < CLASSES && x[i * F + j] > x[i * F + best]) best = j;
    }
    y[i] = best;
  }
}

static int test_mlp(flexflow_config_t cfg) {
  flexflow_model_t model = flexflow_model_create(cfg);
  int dims[2] = {B, F};
  flexflow_tensor_t input = flexflow_tensor_create(model, 2, dims, DT_FLOAT, true);
  CHECK(flexflow_tensor_get_num_dims(input) == 2 && flexflow_tensor_get_dim(input, 0) == F &&
            flexflow_tensor_get_dim(input, 1) == B,
        "tensor dims are reported innermost first");
  flexflow_initializer_t null_init = flexflow_initializer_create_null();
  flexflow_glorot_uniform_initializer_t glorot = flexflow_glorot_uniform_initializer_create(7);
  flexflow_zero_initializer_t zero = flexflow_zero_initializer_create();
  flexflow_initializer_t kinit = {glorot.impl}, binit = {zero.impl};
  flexflow_op_t no_op = {NULL};
  flexflow_tensor_t t = flexflow_model_add_dense(model, input, 64, AC_MODE_RELU, true, DT_FLOAT, no_op, kinit, binit,
                                                 REG_MODE_NONE, 0.f, "fc1");
  t = flexflow_model_add_dense(model, t, CLASSES, AC_MODE_NONE, true, DT_FLOAT, no_op, null_init, null_init,
                               REG_MODE_NONE, 0.f, "fc2");
  t = flexflow_model_add_softmax(model, t, -1, "softmax");
  CHECK(flexflow_tensor_get_dim(t, 0) == CLASSES, "softmax output has %d classes", CLASSES);

  flexflow_op_t fc1 = flexflow_model_get_layer_by_id(model, 0);
  CHECK(flexflow_op_get_num_parameters(fc1) == 2 && flexflow_op_get_num_inputs(fc1) == 1 &&
            flexflow_op_get_num_outputs(fc1) == 1,
        "fc1 has kernel + bias, one input, one output");
  flexflow_op_t last = flexflow_model_get_last_layer(model);
  CHECK(flexflow_tensor_get_owner_op(t).impl == last.impl, "owner op of the output is the last layer");

  flexflow_sgd_optimizer_t sgd = flexflow_sgd_optimizer_create(model, 0.1, 0.9, false, 0.0);
  flexflow_model_set_sgd_optimizer(model, sgd);
  int metrics[1] = {METRICS_ACCURACY};
  flexflow_model_compile(model, LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics, 1, COMP_MODE_TRAINING);
  flexflow_model_init_layers(model);
  printf("device %s\n", flexflow_model_get_device(model));
  flexflow_tensor_t label = flexflow_model_get_label_tensor(model);
  CHECK(flexflow_tensor_get_dim(label, 0) == 1 && flexflow_tensor_get_dim(label, 1) == B,
        "label tensor is [batch, 1]");

  /* weights initialized by the given initializers */
  flexflow_tensor_t bias = flexflow_op_get_parameter_by_id(fc1, 1);
  float b0[64];
  flexflow_parameter_get_weights_float(bias, model, b0);
  int zeros = 1;
  for (int i = 0; i < 64; ++i) zeros &= b0[i] == 0.f;
  CHECK(zeros, "zero initializer on the fc1 bias");

  float* xs = malloc(sizeof(float) * SAMPLES * F);
  int* ys = malloc(sizeof(int) * SAMPLES);
  make_data(xs, ys);
  flexflow_single_dataloader_t dl_x = flexflow_single_dataloader_create2(model, input, xs, SAMPLES, DT_FLOAT);
  flexflow_single_dataloader_t dl_y = flexflow_single_dataloader_create2(model, label, ys, SAMPLES, DT_INT32);
  CHECK(flexflow_single_dataloader_get_num_samples(dl_x) == SAMPLES, "data loader holds %d samples", SAMPLES);

  double t0 = flexflow_get_current_time(cfg);
  float acc = 0.f;
  for (int epoch = 0; epoch < 30; ++epoch) {
    flexflow_single_dataloader_reset(dl_x);
    flexflow_single_dataloader_reset(dl_y);
    flexflow_model_reset_metrics(model);
    for (int it = 0; it < SAMPLES / B; ++it) {
      flexflow_single_dataloader_next_batch(dl_x, model);
      flowflow_single_dataloader_next_batch(dl_y, model);
      flexflow_begin_trace(cfg, 111);
      flexflow_model_forward(model, -1);
      flexflow_model_zero_gradients(model);
      flexflow_model_backward(model, -1);
      flexflow_model_update(model);
      flexflow_end_trace(cfg, 111);
    }
    flexflow_model_compute_metrics(model);
    flexflow_perf_metrics_t pm = flexflow_model_get_perf_metrics(model);
    acc = flexflow_per_metrics_get_accuracy(pm);
    flexflow_per_metrics_destroy(pm);
  }
  double t1 = flexflow_get_current_time(cfg);
  CHECK(acc > 85.f, "MLP learns the synthetic task: last-epoch accuracy %.1f%%", acc);
  CHECK(t1 > t0, "flexflow_get_current_time advances (%.0f us)", t1 - t0);

  /* the output probabilities sum to one; the gradient of a weight exists */
  float probs[B * CLASSES];
  CHECK(flexflow_model_get_output_tensor_float(model, t, probs, false), "read the softmax output");
  float s = 0.f;
  for (int j = 0; j < CLASSES; ++j) s += probs[j];
  CHECK(fabsf(s - 1.f) < 1e-4f, "softmax row sums to 1 (%.6f)", s);
  flexflow_tensor_t kernel = flexflow_op_get_parameter_by_id(fc1, 0);
  float* g = malloc(sizeof(float) * F * 64);
  CHECK(flexflow_tensor_get_tensor_float(kernel, model, g, true), "read the fc1 kernel gradient");

  /* raw pointers are the slot itself (zero copy) */
  float* raw = flexflow_tensor_get_raw_ptr_float(input, model, cfg);
  CHECK(raw && raw[0] == xs[((SAMPLES / B - 1) * B) * F], "raw pointer shows the last batch");

  /* errors are reported, not fatal */
  int bad_dims[2] = {3, 3};
  CHECK(!flexflow_tensor_set_tensor_float(input, model, 2, bad_dims, xs) &&
            strstr(flexflow_runtime_last_error(), "mismatch") != NULL,
        "size mismatch is reported: %s", flexflow_runtime_last_error());

  flexflow_sgd_optimizer_set_lr(sgd, 0.01);
  flexflow_model_print_layers(model, 0);
  flexflow_single_dataloader_destroy(dl_x);
  flexflow_single_dataloader_destroy(dl_y);
  flexflow_sgd_optimizer_destroy(sgd);
  flexflow_glorot_uniform_initializer_destroy(glorot);
  flexflow_zero_initializer_destroy(zero);
  flexflow_model_destroy(model);
  free(xs);
  free(ys);
  free(g);
  return 0;
}

static int test_cnn(flexflow_config_t cfg) {
  enum { N = 8, C = 3, H = 8, W = 8 };
  flexflow_model_t model = flexflow_model_create(cfg);
  int dims[4] = {N, C, H, W};
  flexflow_tensor_t x = flexflow_tensor_create(model, 4, dims, DT_FLOAT, true);
  flexflow_initializer_t null_init = flexflow_initializer_create_null();
  flexflow_op_t no_op = {NULL};
  flexflow_tensor_t t = flexflow_model_add_conv2d(model, x, 4, 3, 3, 1, 1, 1, 1, AC_MODE_RELU, 1, true, no_op,
                                                  null_init, null_init, "conv");
  t = flexflow_model_add_batch_norm(model, t, true, "bn");
  t = flexflow_model_add_pool2d(model, t, 2, 2, 2, 2, 0, 0, POOL_MAX, AC_MODE_NONE, "pool");
  CHECK(flexflow_tensor_get_dim(t, 0) == 4 && flexflow_tensor_get_dim(t, 1) == 4 &&
            flexflow_tensor_get_dim(t, 2) == 4 && flexflow_tensor_get_dim(t, 3) == N,
        "conv/pool output is N x 4 x 4 x 4");
  t = flexflow_model_add_flat(model, t, "flat");
  t = flexflow_model_add_dense(model, t, 3, AC_MODE_NONE, true, DT_FLOAT, no_op, null_init, null_init,
                               REG_MODE_NONE, 0.f, "head");
  t = flexflow_model_add_softmax(model, t, -1, "sm");
  flexflow_adam_optimizer_t adam = flexflow_adam_optimizer_create(model, 0.01, 0.9, 0.999, 0.0, 1e-8);
  flexflow_model_set_adam_optimizer(model, adam);
  int metrics[1] = {METRICS_ACCURACY};
  flexflow_model_compile(model, LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics, 1, COMP_MODE_TRAINING);
  printf("cnn device %s\n", flexflow_model_get_device(model));
  float img[N * C * H * W];
  int lab[N];
  for (int i = 0; i < N * C * H * W; ++i) img[i] = sinf(0.37f * (float)i);
  for (int i = 0; i < N; ++i) lab[i] = i % 3;
  int ldims[2] = {N, 1};
  flexflow_tensor_set_tensor_float(x, model, 4, dims, img);
  flexflow_tensor_set_tensor_int(flexflow_model_get_label_tensor(model), model, 2, ldims, lab);
  flexflow_op_t conv = flexflow_model_get_layer_by_id(model, 0);
  flexflow_tensor_t k = flexflow_op_get_parameter_by_id(conv, 0);
  float before[4 * 3 * 3 * 3], after[4 * 3 * 3 * 3];
  flexflow_parameter_get_weights_float(k, model, before);
  float first = 0.f, last = 0.f;
  for (int step = 0; step < 40; ++step) {
    flexflow_model_reset_metrics(model);
    flexflow_model_forward(model, -1);
    flexflow_model_backward(model, -1);
    flexflow_model_update(model);
    flexflow_perf_metrics_t pm = flexflow_model_get_perf_metrics(model);
    if (step == 0) first = flexflow_per_metrics_get_accuracy(pm);
    last = flexflow_per_metrics_get_accuracy(pm);
    flexflow_per_metrics_destroy(pm);
  }
  flexflow_parameter_get_weights_float(k, model, after);
  CHECK(memcmp(before, after, sizeof(before)) != 0, "conv kernel trained");
  CHECK(last >= first && last == 100.f, "CNN memorizes 8 images (accuracy %.0f%% -> %.0f%%)", first, last);
  /* a single operator forward */
  flexflow_op_forward(conv, model);
  CHECK(flexflow_runtime_last_error()[0] == '\0' || strstr(flexflow_runtime_last_error(), "mismatch"),
        "op forward runs");
  flexflow_adam_optimizer_destroy(adam);
  flexflow_model_destroy(model);
  return 0;
}

/* three SGD steps of a two-layer MLP (tanh, sigmoid heads; MSE), the
 * trained weights printed with full precision: the GPU and the CPU backings
 * must agree (tests/test_runtime_c_gpu.py runs this twice) */
static void test_parity(flexflow_config_t cfg) {
  enum { PB = 16, PF = 24, PH = 40, PO = 3 };
  flexflow_model_t model = flexflow_model_create(cfg);
  int dims[2] = {PB, PF};
  flexflow_tensor_t x = flexflow_tensor_create(model, 2, dims, DT_FLOAT, true);
  flexflow_initializer_t null_init = flexflow_initializer_create_null();
  flexflow_op_t no_op = {NULL};
  flexflow_tensor_t t = flexflow_model_add_dense(model, x, PH, AC_MODE_TANH, true, DT_FLOAT, no_op, null_init,
                                                 null_init, REG_MODE_NONE, 0.f, "p1");
  t = flexflow_model_add_dense(model, t, PO, AC_MODE_SIGMOID, true, DT_FLOAT, no_op, null_init, null_init,
                               REG_MODE_NONE, 0.f, "p2");
  flexflow_adam_optimizer_t adam = flexflow_adam_optimizer_create(model, 0.01, 0.9, 0.999, 0.0, 1e-8);
  flexflow_model_set_adam_optimizer(model, adam);
  int metrics[1] = {METRICS_MEAN_SQUARED_ERROR};
  flexflow_model_compile(model, LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, metrics, 1, COMP_MODE_TRAINING);
  float xs[PB * PF], ys[PB * PO];
  for (int i = 0; i < PB * PF; ++i) xs[i] = cosf(0.11f * (float)i);
  for (int i = 0; i < PB * PO; ++i) ys[i] = 0.5f + 0.4f * sinf(0.3f * (float)i);
  int ldims[2] = {PB, PO};
  flexflow_tensor_set_tensor_float(x, model, 2, dims, xs);
  flexflow_tensor_set_tensor_float(flexflow_model_get_label_tensor(model), model, 2, ldims, ys);
  for (int step = 0; step < 3; ++step) {
    flexflow_model_forward(model, -1);
    flexflow_model_zero_gradients(model);
    flexflow_model_backward(model, -1);
    flexflow_model_update(model);
  }
  flexflow_op_t l2 = flexflow_model_get_layer_by_id(model, 1);
  float w[PH * PO];
  flexflow_parameter_get_weights_float(flexflow_op_get_parameter_by_id(l2, 0), model, w);
  double sum = 0.0, asum = 0.0;
  for (int i = 0; i < PH * PO; ++i) {
    sum += w[i];
    asum += fabs(w[i]);
  }
  printf("parity device %s w2_sum %.9g w2_abs %.9g w2_0 %.9g\n", flexflow_model_get_device(model), sum, asum, w[0]);
  flexflow_adam_optimizer_destroy(adam);
  flexflow_model_destroy(model);
}

/* the CNN path (conv + relu, batch norm, max / avg pooling, flat, dense,
 * softmax + cross-entropy) for three Adam steps, the conv kernel printed:
 * GPU and CPU backings must agree (tests/test_runtime_c_gpu.py) */
static void test_parity_cnn(flexflow_config_t cfg) {
  enum { N = 4, C = 3, H = 10, W = 10 };
  flexflow_model_t model = flexflow_model_create(cfg);
  int dims[4] = {N, C, H, W};
  flexflow_tensor_t x = flexflow_tensor_create(model, 4, dims, DT_FLOAT, true);
  flexflow_initializer_t null_init = flexflow_initializer_create_null();
  flexflow_op_t no_op = {NULL};
  flexflow_tensor_t t = flexflow_model_add_conv2d(model, x, 6, 3, 3, 1, 1, 1, 1, AC_MODE_RELU, 1, true, no_op,
                                                  null_init, null_init, "pc1");
  t = flexflow_model_add_batch_norm(model, t, true, "pbn");
  t = flexflow_model_add_pool2d(model, t, 2, 2, 2, 2, 0, 0, POOL_MAX, AC_MODE_NONE, "ppool");
  t = flexflow_model_add_conv2d(model, t, 4, 3, 3, 2, 2, 1, 1, AC_MODE_TANH, 1, true, no_op, null_init, null_init,
                                "pc2");
  t = flexflow_model_add_pool2d(model, t, 2, 2, 1, 1, 1, 1, POOL_AVG, AC_MODE_NONE, "pavg");
  t = flexflow_model_add_flat(model, t, "pflat");
  t = flexflow_model_add_dense(model, t, 3, AC_MODE_NONE, true, DT_FLOAT, no_op, null_init, null_init,
                               REG_MODE_NONE, 0.f, "phead");
  t = flexflow_model_add_softmax(model, t, -1, "psm");
  flexflow_adam_optimizer_t adam = flexflow_adam_optimizer_create(model, 0.01, 0.9, 0.999, 0.0, 1e-8);
  flexflow_model_set_adam_optimizer(model, adam);
  int metrics[1] = {METRICS_ACCURACY};
  flexflow_model_compile(model, LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics, 1, COMP_MODE_TRAINING);
  float img[N * C * H * W];
  int lab[N];
  for (int i = 0; i < N * C * H * W; ++i) img[i] = sinf(0.23f * (float)i) + 0.1f * cosf(0.05f * (float)i);
  for (int i = 0; i < N; ++i) lab[i] = i % 3;
  int ldims[2] = {N, 1};
  flexflow_tensor_set_tensor_float(x, model, 4, dims, img);
  flexflow_tensor_set_tensor_int(flexflow_model_get_label_tensor(model), model, 2, ldims, lab);
  for (int step = 0; step < 3; ++step) {
    flexflow_model_forward(model, -1);
    flexflow_model_zero_gradients(model);
    flexflow_model_backward(model, -1);
    flexflow_model_update(model);
  }
  flexflow_op_t c1 = flexflow_model_get_layer_by_id(model, 0);
  float w[6 * 3 * 3 * 3];
  flexflow_parameter_get_weights_float(flexflow_op_get_parameter_by_id(c1, 0), model, w);
  double sum = 0.0, asum = 0.0;
  for (int i = 0; i < 6 * 27; ++i) {
    sum += w[i];
    asum += fabs(w[i]);
  }
  printf("parity_cnn device %s w_sum %.9g w_abs %.9g w_0 %.9g\n", flexflow_model_get_device(model), sum, asum, w[0]);
  flexflow_adam_optimizer_destroy(adam);
  flexflow_model_destroy(model);
}


/* a 2-layer BERT-style encoder through the C API (embedding, multi-head
 * attention with biases, residual adds, layer norms, GELU FFN with dropout,
 * split + concat, a batch-matmul side branch over a reshaped view, the
 * vocabulary head + softmax cross-entropy) for three Adam steps: the GPU
 * backing (production kernels) and the CPU backing must agree
 * (tests/test_runtime_c_gpu.py) */
static void test_parity_bert(flexflow_config_t cfg) {
  enum { BB = 4, S = 16, V = 40, D = 32, HEADS = 4, FF = 64 };
  flexflow_model_t model = flexflow_model_create(cfg);
  int dims[2] = {BB, S};
  flexflow_tensor_t tok = flexflow_tensor_create(model, 2, dims, DT_INT32, false);
  flexflow_initializer_t null_init = flexflow_initializer_create_null();
  flexflow_op_t no_op = {NULL};
  flexflow_tensor_t x = flexflow_model_add_embedding(model, tok, V, D, AGGR_MODE_NONE, no_op, null_init, "emb");
  int ln_axes[1] = {-1};
  for (int l = 0; l < 2; ++l) {
    char nm[32];
    snprintf(nm, sizeof nm, "attn%d", l);
    flexflow_tensor_t a = flexflow_model_add_multihead_attention(model, x, x, x, D, HEADS, D / HEADS, D / HEADS, 0.f,
                                                                 true, false, false, null_init, nm);
    x = flexflow_model_add_layer_norm(model, flexflow_model_add_add(model, x, a, false, NULL), 1, ln_axes, true, 1e-5f,
                                      NULL);
    flexflow_tensor_t f = flexflow_model_add_dense(model, x, FF, AC_MODE_GELU, true, DT_FLOAT, no_op, null_init,
                                                   null_init, REG_MODE_NONE, 0.f, NULL);
    f = flexflow_model_add_dropout(model, f, 0.1f, 3, NULL);
    f = flexflow_model_add_dense(model, f, D, AC_MODE_NONE, true, DT_FLOAT, no_op, null_init, null_init,
                                 REG_MODE_NONE, 0.f, NULL);
    if (l == 0) {   /* split the FFN output in two along the features and put it back */
      flexflow_tensor_t halves[2];
      int sizes[2] = {D / 2, D / 2};
      flexflow_model_add_split(model, f, 2, halves, sizes, 2, NULL);
      f = flexflow_model_add_concat(model, 2, halves, 2, NULL);
    } else {        /* x [B,S,D] @ view(x) [B,D,S] -> [B,S,S] -> dense back to D, added in */
      int rs[3] = {BB, D, S};
      flexflow_tensor_t xr = flexflow_model_add_reshape(model, x, 3, rs, NULL);
      flexflow_tensor_t z = flexflow_model_add_batch_matmul(model, x, xr, -1, -1);
      z = flexflow_model_add_dense(model, z, D, AC_MODE_NONE, false, DT_FLOAT, no_op, null_init, null_init,
                                   REG_MODE_NONE, 0.f, NULL);
      f = flexflow_model_add_add(model, f, flexflow_model_add_scalar_multiply(model, z, 0.1f, false, NULL), false,
                                 NULL);
    }
    x = flexflow_model_add_layer_norm(model, flexflow_model_add_add(model, x, f, false, NULL), 1, ln_axes, true, 1e-5f,
                                      NULL);
  }
  flexflow_tensor_t logits = flexflow_model_add_dense(model, x, V, AC_MODE_NONE, true, DT_FLOAT, no_op, null_init,
                                                      null_init, REG_MODE_NONE, 0.f, "head");
  flexflow_model_add_softmax(model, logits, -1, "sm");
  flexflow_adam_optimizer_t adam = flexflow_adam_optimizer_create(model, 0.005, 0.9, 0.999, 0.0, 1e-8);
  flexflow_model_set_adam_optimizer(model, adam);
  int metrics[1] = {METRICS_ACCURACY};
  flexflow_model_compile(model, LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics, 1, COMP_MODE_TRAINING);
  int ids[BB * S], lab[BB * S];
  for (int i = 0; i < BB * S; ++i) {
    ids[i] = (i * 7 + 3) % V;
    lab[i] = (i * 5 + 1) % V;
  }
  flexflow_tensor_set_tensor_int(tok, model, 2, dims, ids);
  int ldims[3] = {BB, S, 1};
  flexflow_tensor_set_tensor_int(flexflow_model_get_label_tensor(model), model, 3, ldims, lab);
  for (int step = 0; step < 3; ++step) {
    flexflow_model_forward(model, -1);
    flexflow_model_zero_gradients(model);
    flexflow_model_backward(model, -1);
    flexflow_model_update(model);
  }
  static float we[V * D], wa[4096];
  flexflow_parameter_get_weights_float(flexflow_op_get_parameter_by_id(flexflow_model_get_layer_by_id(model, 0), 0),
                                       model, we);
  flexflow_parameter_get_weights_float(flexflow_op_get_parameter_by_id(flexflow_model_get_layer_by_id(model, 1), 0),
                                       model, wa);
  double se = 0.0, sa = 0.0, aa = 0.0;
  for (int i = 0; i < V * D; ++i) se += we[i];
  for (int i = 0; i < 4096; ++i) {
    sa += wa[i];
    aa += fabs(wa[i]);
  }
  printf("parity_bert device %s emb_sum %.9g attn_sum %.9g attn_abs %.9g attn_0 %.9g\n",
         flexflow_model_get_device(model), se, sa, aa, wa[0]);
  flexflow_adam_optimizer_destroy(adam);
  flexflow_model_destroy(model);
}

static void test_configs(void) {
  char* argv[] = {"prog", "-b", "32", "--epochs", "3", "--arch-mlp-bot", "13-512-256-64", "--arch-embedding-size",
                  "1000-1000", "--arch-sparse-feature-size", "64", "--dataset", "/tmp/x.h5", "-ll:gpu", "8"};
  begin_flexflow_task(15, argv);
  flexflow_config_t cfg = flexflow_config_create();
  CHECK(flexflow_config_get_batch_size(cfg) == 32 && flexflow_config_get_epochs(cfg) == 3 &&
            flexflow_config_get_workers_per_node(cfg) == 8 && flexflow_config_get_num_nodes(cfg) == 1,
        "FFConfig parses -b / --epochs / -ll:gpu");
  CHECK(flexflow_config_get_enable_control_replication(cfg) && flexflow_config_get_python_data_loader_type(cfg) == 2,
        "FFConfig defaults");
  flexflow_dlrm_config_t d = flexflow_dlrm_config_create();
  int* bot = flexflow_dlrm_config_get_mlp_bot(d);
  int* emb = flexflow_dlrm_config_get_embedding_size(d);
  int* top = flexflow_dlrm_config_get_mlp_top(d);
  CHECK(bot[0] == 4 && bot[1] == 13 && bot[4] == 64 && emb[0] == 2 && emb[1] == 1000 && top[0] == 2 &&
            flexflow_dlrm_config_get_sparse_feature_size(d) == 64 &&
            strcmp(flexflow_dlrm_config_get_arch_interaction_op(d), "cat") == 0 &&
            strcmp(flexflow_dlrm_config_get_dataset_path(d), "/tmp/x.h5") == 0,
        "DLRMConfig parses the reference flags");
  flexflow_net_config_t n = flexflow_net_config_create();
  CHECK(strcmp(flexflow_net_config_get_dataset_path(n), "/tmp/x.h5") == 0, "NetConfig parses --dataset");
  flexflow_net_config_destroy(n);
  flexflow_dlrm_config_destroy(d);
  flexflow_config_destroy(cfg);
  finish_flexflow_task();
}

int main(int argc, char** argv) {
  register_c_custom_tasks();
  test_configs();
  begin_flexflow_task(argc, argv);
  flexflow_config_t cfg = flexflow_config_create();
  flexflow_config_parse_args_default(cfg);
  test_mlp(cfg);
  test_cnn(cfg);
  test_parity(cfg);
  test_parity_cnn(cfg);
  test_parity_bert(cfg);
  flexflow_config_destroy(cfg);
  finish_flexflow_task();
  printf("%s (%d failures)\n", failures ? "FAILED" : "PASSED", failures);
  return failures ? 1 : 0;
}
