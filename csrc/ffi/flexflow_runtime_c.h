/* Legacy FFModel runtime C API (libflexflow_runtime_c.so).
 *
 * The reference ships two C APIs that cannot be linked into one program
 * (both define flexflow_tensor_create & co.): the graph-building FFI of its
 * new libraries (lib/pcg/ffi, lib/compiler/ffi -> csrc/ffi/flexflow_c.h
 * here) and the FFModel runtime API its Python package drove through cffi
 * (python/flexflow_c.h).  This header is the second one, with the same
 * function names, argument lists and enum values, so a C host written
 * against it builds and trains unchanged.
 *
 * What runs underneath: the model is a ComputationGraph (csrc/ffcore); on
 * compile() it is handed to the native LocalTrainingBacking
 * (csrc/ffcore/src/local_exec.cc, the lib/local-execution counterpart),
 * which runs forward / loss + metrics / backward / SGD-or-Adam on the host.
 * Multi-GPU training stays with the per-rank Python executor (RCCL); this
 * API is the single-process runtime surface.  Legion-only calls (inline
 * map / unmap, trace begin / end, task registration) are accepted and do
 * what they mean here: nothing to map, traces are counted.
 *
 * Handles are {void* impl} structs passed by value, released with the
 * matching *_destroy.  Errors (an unknown layer, a shape mismatch, an
 * operator the host backing does not execute) print one line to stderr and
 * return a null handle / false; flexflow_runtime_last_error() has the text.
 */
#ifndef FLEXFLOW_RUNTIME_C_H
#define FLEXFLOW_RUNTIME_C_H

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FF_RT_API __attribute__((visibility("default")))
#define FF_RT_HANDLE(T) \
  typedef struct T {    \
    void* impl;         \
  } T

FF_RT_HANDLE(flexflow_config_t);
FF_RT_HANDLE(flexflow_model_t);
FF_RT_HANDLE(flexflow_tensor_t);
FF_RT_HANDLE(flexflow_parallel_tensor_t);
FF_RT_HANDLE(flexflow_sgd_optimizer_t);
FF_RT_HANDLE(flexflow_adam_optimizer_t);
FF_RT_HANDLE(flexflow_initializer_t);
FF_RT_HANDLE(flexflow_glorot_uniform_initializer_t);
FF_RT_HANDLE(flexflow_zero_initializer_t);
FF_RT_HANDLE(flexflow_uniform_initializer_t);
FF_RT_HANDLE(flexflow_norm_initializer_t);
FF_RT_HANDLE(flexflow_op_t);
FF_RT_HANDLE(flexflow_perf_metrics_t);
FF_RT_HANDLE(flexflow_net_config_t);
FF_RT_HANDLE(flexflow_dlrm_config_t);
FF_RT_HANDLE(flexflow_dataloader_4d_t);
FF_RT_HANDLE(flexflow_dataloader_2d_t);
FF_RT_HANDLE(flexflow_single_dataloader_t);

/* enum values of the reference's flexflow/ffconst.h (python/flexflow/type.py) */
enum ActiMode { AC_MODE_NONE = 10, AC_MODE_RELU = 11, AC_MODE_SIGMOID = 12, AC_MODE_TANH = 13, AC_MODE_GELU = 14 };
enum RegularizerMode { REG_MODE_NONE = 17, REG_MODE_L1 = 18, REG_MODE_L2 = 19 };
enum AggrMode { AGGR_MODE_NONE = 20, AGGR_MODE_SUM = 21, AGGR_MODE_AVG = 22 };
enum PoolType { POOL_MAX = 30, POOL_AVG = 31 };
enum DataType {
  DT_BOOLEAN = 40, DT_INT32 = 41, DT_INT64 = 42, DT_HALF = 43, DT_FLOAT = 44, DT_DOUBLE = 45, DT_NONE = 49
};
enum LossType {
  LOSS_CATEGORICAL_CROSSENTROPY = 50,
  LOSS_SPARSE_CATEGORICAL_CROSSENTROPY = 51,
  LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE = 52,
  LOSS_MEAN_SQUARED_ERROR_SUM_REDUCE = 53,
  LOSS_IDENTITY = 54
};
enum CompMode { COMP_MODE_TRAINING = 70, COMP_MODE_INFERENCE = 71 };
enum ParameterSyncType { PARAMETER_SYNC_NONE = 80, PARAMETER_SYNC_PS = 81, PARAMETER_SYNC_NCCL = 82 };
enum MetricsType {
  METRICS_ACCURACY = 1001,
  METRICS_CATEGORICAL_CROSSENTROPY = 1002,
  METRICS_SPARSE_CATEGORICAL_CROSSENTROPY = 1004,
  METRICS_MEAN_SQUARED_ERROR = 1008,
  METRICS_ROOT_MEAN_SQUARED_ERROR = 1016,
  METRICS_MEAN_ABSOLUTE_ERROR = 1032
};

FF_RT_API const char* flexflow_runtime_last_error(void);
/* where a compiled model trains: "gpu:<n>" (the HIP backing) or "cpu" (with
 * the reason the GPU backing was not taken, e.g. "cpu (no GPU visible)") */
FF_RT_API const char* flexflow_model_get_device(flexflow_model_t model);

/* ---- FFConfig ---------------------------------------------------------- */
FF_RT_API flexflow_config_t flexflow_config_create(void);
FF_RT_API void flexflow_config_destroy(flexflow_config_t handle);
/* the reference's command-line flags: -b / --batch-size, -e / --epochs,
 * --lr, --wd, --nodes, -ll:gpu (workers per node), --only-data-parallel, ...
 * (unknown flags are ignored, as the reference's parser does) */
FF_RT_API void flexflow_config_parse_args(flexflow_config_t handle, char** argv, int argc);
FF_RT_API void flexflow_config_parse_args_default(flexflow_config_t handle);
FF_RT_API int flexflow_config_get_batch_size(flexflow_config_t handle);
FF_RT_API int flexflow_config_get_workers_per_node(flexflow_config_t handle);
FF_RT_API int flexflow_config_get_num_nodes(flexflow_config_t handle);
FF_RT_API int flexflow_config_get_epochs(flexflow_config_t handle);
FF_RT_API bool flexflow_config_get_enable_control_replication(flexflow_config_t handle);
FF_RT_API int flexflow_config_get_python_data_loader_type(flexflow_config_t handle);

/* ---- FFModel ----------------------------------------------------------- */
FF_RT_API flexflow_model_t flexflow_model_create(flexflow_config_t config);
FF_RT_API void flexflow_model_destroy(flexflow_model_t handle);
FF_RT_API void flexflow_model_reset_metrics(flexflow_model_t handle);
FF_RT_API void flexflow_model_init_layers(flexflow_model_t handle);
FF_RT_API void flexflow_model_prefetch(flexflow_model_t handle);
FF_RT_API void flexflow_model_forward(flexflow_model_t handle, int seq_length);
FF_RT_API void flexflow_model_backward(flexflow_model_t handle, int seq_length);
FF_RT_API void flexflow_model_compute_metrics(flexflow_model_t handle);
FF_RT_API void flexflow_model_update(flexflow_model_t handle);
FF_RT_API void flexflow_model_compile(flexflow_model_t handle, enum LossType loss_type, int* metrics, int nb_metrics,
                                      enum CompMode comp_mode);
FF_RT_API flexflow_tensor_t flexflow_model_get_label_tensor(flexflow_model_t handle);
FF_RT_API void flexflow_model_zero_gradients(flexflow_model_t handle);

/* element-wise */
FF_RT_API flexflow_tensor_t flexflow_model_add_exp(flexflow_model_t handle, const flexflow_tensor_t x, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_sin(flexflow_model_t handle, const flexflow_tensor_t x, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_cos(flexflow_model_t handle, const flexflow_tensor_t x, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_add(flexflow_model_t handle, const flexflow_tensor_t x,
                                                   const flexflow_tensor_t y, bool inplace_a, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_subtract(flexflow_model_t handle, const flexflow_tensor_t x,
                                                        const flexflow_tensor_t y, bool inplace_a, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_multiply(flexflow_model_t handle, const flexflow_tensor_t x,
                                                        const flexflow_tensor_t y, bool inplace_a, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_divide(flexflow_model_t handle, const flexflow_tensor_t x,
                                                      const flexflow_tensor_t y, bool inplace_a, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_max(flexflow_model_t handle, const flexflow_tensor_t x,
                                                   const flexflow_tensor_t y, bool inplace_a, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_min(flexflow_model_t handle, const flexflow_tensor_t x,
                                                   const flexflow_tensor_t y, bool inplace_a, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_reduce_sum(flexflow_model_t handle, const flexflow_tensor_t input,
                                                          int* axes, int n, bool keepdims, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_rsqrt(flexflow_model_t handle, const flexflow_tensor_t input,
                                                     const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_pow(flexflow_model_t handle, const flexflow_tensor_t input,
                                                   const float exponent, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_mean(flexflow_model_t handle, const flexflow_tensor_t input, int* dims,
                                                    int n, bool keepdims, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_relu(flexflow_model_t handle, const flexflow_tensor_t input,
                                                    bool inplace, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_scalar_multiply(flexflow_model_t handle, const flexflow_tensor_t input,
                                                               const float scalar, bool inplace, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_scalar_add(flexflow_model_t handle, const flexflow_tensor_t input,
                                                          const float scalar, bool inplace, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_scalar_sub(flexflow_model_t handle, const flexflow_tensor_t input,
                                                          const float scalar, bool inplace, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_scalar_truediv(flexflow_model_t handle, const flexflow_tensor_t input,
                                                              const float scalar, bool inplace, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_gelu(flexflow_model_t handle, const flexflow_tensor_t input,
                                                    const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_identity(flexflow_model_t handle, const flexflow_tensor_t input,
                                                        const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_sigmoid(flexflow_model_t handle, const flexflow_tensor_t input,
                                                       const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_tanh(flexflow_model_t handle, const flexflow_tensor_t input,
                                                    const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_elu(flexflow_model_t handle, const flexflow_tensor_t input,
                                                   bool inplace, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_dropout(flexflow_model_t handle, const flexflow_tensor_t input,
                                                       float rate, unsigned long long seed, const char* name);

/* layers with weights / structure */
FF_RT_API flexflow_tensor_t flexflow_model_add_conv2d(flexflow_model_t handle, const flexflow_tensor_t input,
                                                      int out_channels, int kernel_h, int kernel_w, int stride_h,
                                                      int stride_w, int padding_h, int padding_w,
                                                      enum ActiMode activation, int groups, bool use_bias,
                                                      flexflow_op_t shared_op,
                                                      flexflow_initializer_t kernel_initializer,
                                                      flexflow_initializer_t bias_initializer, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_embedding(flexflow_model_t handle, const flexflow_tensor_t input,
                                                         int num_entires, int out_dim, enum AggrMode aggr,
                                                         flexflow_op_t shared_op,
                                                         flexflow_initializer_t kernel_initializer, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_pool2d(flexflow_model_t handle, flexflow_tensor_t input, int kernel_h,
                                                      int kernel_w, int stride_h, int stride_w, int padding_h,
                                                      int padding_w, enum PoolType type, enum ActiMode activation,
                                                      const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_batch_norm(flexflow_model_t handle, const flexflow_tensor_t input,
                                                          bool relu, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_layer_norm(flexflow_model_t handle, const flexflow_tensor_t input,
                                                          int n, int* axes, bool elementwise_affine, float eps,
                                                          const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_batch_matmul(flexflow_model_t handle, const flexflow_tensor_t a,
                                                            const flexflow_tensor_t b, int a_seq_length_dim,
                                                            int b_seq_length_dim);
FF_RT_API flexflow_tensor_t flexflow_model_add_dense(flexflow_model_t handle, const flexflow_tensor_t input,
                                                     int out_dim, enum ActiMode activation, bool use_bias,
                                                     enum DataType data_type, flexflow_op_t shared_op,
                                                     flexflow_initializer_t kernel_initializer,
                                                     flexflow_initializer_t bias_initializer,
                                                     enum RegularizerMode kernel_reg_type, float kernel_reg_lambda,
                                                     const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_concat(flexflow_model_t handle, int n, flexflow_tensor_t* input,
                                                      int axis, const char* name);
FF_RT_API void flexflow_model_add_split(flexflow_model_t handle, flexflow_tensor_t input, int n,
                                        flexflow_tensor_t* outputs, int* split, int axis, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_flat(flexflow_model_t handle, flexflow_tensor_t input,
                                                    const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_gather(flexflow_model_t handle, const flexflow_tensor_t input,
                                                      const flexflow_tensor_t index, int dim, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_softmax(flexflow_model_t handle, const flexflow_tensor_t input, int dim,
                                                       const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_transpose(flexflow_model_t handle, const flexflow_tensor_t input, int n,
                                                         int* perm, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_reshape(flexflow_model_t handle, const flexflow_tensor_t input, int n,
                                                       int* shape, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_reverse(flexflow_model_t handle, const flexflow_tensor_t input,
                                                       int axis, const char* name);
FF_RT_API flexflow_tensor_t flexflow_model_add_multihead_attention(
    flexflow_model_t handle, const flexflow_tensor_t query, const flexflow_tensor_t key,
    const flexflow_tensor_t value, int embed_dim, int num_heads, int kdim, int vdim, float dropout, bool bias,
    bool add_bias_kv, bool add_zero_attn, flexflow_initializer_t kernel_initializer, const char* name);

FF_RT_API void flexflow_model_set_sgd_optimizer(flexflow_model_t handle, flexflow_sgd_optimizer_t optimizer);
FF_RT_API void flexflow_model_set_adam_optimizer(flexflow_model_t handle, flexflow_adam_optimizer_t optimizer);
FF_RT_API void flexflow_model_print_layers(flexflow_model_t handle, int id);
FF_RT_API flexflow_op_t flexflow_model_get_layer_by_id(flexflow_model_t handle, int layer_id);
FF_RT_API flexflow_op_t flexflow_model_get_last_layer(flexflow_model_t handle);
FF_RT_API flexflow_tensor_t flexflow_model_get_parameter_by_id(flexflow_model_t handle, int layer_id);
FF_RT_API flexflow_perf_metrics_t flexflow_model_get_perf_metrics(flexflow_model_t handle);
FF_RT_API bool flexflow_model_get_output_tensor_float(flexflow_model_t model, flexflow_tensor_t handle, float* data,
                                                      bool get_gradients);

/* ---- Tensor ------------------------------------------------------------ */
FF_RT_API flexflow_tensor_t flexflow_tensor_create(flexflow_model_t model, int num_dims, const int* dims,
                                                   enum DataType data_type, bool create_grad);
FF_RT_API void flexflow_tensor_map(flexflow_model_t model, flexflow_tensor_t tensor, flexflow_op_t op);
FF_RT_API flexflow_tensor_t flexflow_constant_create(flexflow_model_t model, int num_dims, const int* dims,
                                                     float value, enum DataType data_type);
FF_RT_API void flexflow_tensor_destroy(flexflow_tensor_t handle);
FF_RT_API void flexflow_tensor_inline_map(flexflow_tensor_t handle, flexflow_model_t model, flexflow_config_t config);
FF_RT_API void flexflow_tensor_inline_unmap(flexflow_tensor_t handle, flexflow_model_t model,
                                            flexflow_config_t config);
FF_RT_API float* flexflow_tensor_get_raw_ptr_float(flexflow_tensor_t handle, flexflow_model_t model,
                                                   flexflow_config_t config);
FF_RT_API int32_t* flexflow_tensor_get_raw_ptr_int32(flexflow_tensor_t handle, flexflow_model_t model,
                                                     flexflow_config_t config);
FF_RT_API int flexflow_tensor_get_num_dims(flexflow_tensor_t handle);
/* legion_axis counts from the innermost dimension, as in the reference */
FF_RT_API int flexflow_tensor_get_dim(flexflow_tensor_t handle, int legion_axis);
FF_RT_API int* flexflow_tensor_get_dims(flexflow_tensor_t handle);
FF_RT_API int flexflow_tensor_get_data_type(flexflow_tensor_t handle);
FF_RT_API flexflow_op_t flexflow_tensor_get_owner_op(flexflow_tensor_t handle);
FF_RT_API void flexflow_tensor_attach_raw_ptr(flexflow_tensor_t handle, flexflow_model_t model,
                                              flexflow_config_t config, void* raw_ptr, bool column_major);
FF_RT_API void flexflow_tensor_detach_raw_ptr(flexflow_tensor_t handle, flexflow_model_t model,
                                              flexflow_config_t config);
FF_RT_API bool flexflow_tensor_is_mapped(flexflow_tensor_t handle);
FF_RT_API bool flexflow_tensor_set_tensor_float(flexflow_tensor_t handle, flexflow_model_t model, int num_dim,
                                                int* dims, const float* data);
FF_RT_API bool flexflow_tensor_get_tensor_float(flexflow_tensor_t handle, flexflow_model_t model, float* data,
                                                bool get_gradients);
FF_RT_API bool flexflow_tensor_set_tensor_int(flexflow_tensor_t handle, flexflow_model_t model, int num_dim, int* dims,
                                              const int* data);
FF_RT_API bool flexflow_tensor_get_tensor_int(flexflow_tensor_t handle, flexflow_model_t model, int* data,
                                              bool get_gradients);
FF_RT_API bool flexflow_tensor_set_tensor_int64(flexflow_tensor_t handle, flexflow_model_t model, int num_dim,
                                                int* dims, const int64_t* data, enum ParameterSyncType comm_type);
FF_RT_API bool flexflow_tensor_get_tensor_int64(flexflow_tensor_t handle, flexflow_model_t model, int64_t* data,
                                                bool get_gradients);
FF_RT_API bool flexflow_parameter_set_weights_float(flexflow_tensor_t handle, flexflow_model_t model, int num_dim,
                                                    int* dims, const float* data);
FF_RT_API bool flexflow_parameter_get_weights_float(flexflow_tensor_t handle, flexflow_model_t model, float* data);

/* ---- Optimizers / initializers / metrics ------------------------------- */
FF_RT_API flexflow_sgd_optimizer_t flexflow_sgd_optimizer_create(flexflow_model_t model, double lr, double momentum,
                                                                 bool nesterov, double weight_decay);
FF_RT_API void flexflow_sgd_optimizer_destroy(flexflow_sgd_optimizer_t handle);
FF_RT_API void flexflow_sgd_optimizer_set_lr(flexflow_sgd_optimizer_t handle, double lr);
FF_RT_API flexflow_adam_optimizer_t flexflow_adam_optimizer_create(flexflow_model_t model, double alpha, double beta1,
                                                                   double beta2, double weight_decay, double epsilon);
FF_RT_API void flexflow_adam_optimizer_destroy(flexflow_adam_optimizer_t handle);
FF_RT_API void flexflow_adam_optimizer_set_lr(flexflow_adam_optimizer_t handle, double lr);

FF_RT_API flexflow_initializer_t flexflow_initializer_create_null(void);
FF_RT_API flexflow_glorot_uniform_initializer_t flexflow_glorot_uniform_initializer_create(int seed);
FF_RT_API void flexflow_glorot_uniform_initializer_destroy(flexflow_glorot_uniform_initializer_t handle);
FF_RT_API flexflow_zero_initializer_t flexflow_zero_initializer_create(void);
FF_RT_API void flexflow_zero_initializer_destroy(flexflow_zero_initializer_t handle);
FF_RT_API flexflow_uniform_initializer_t flexflow_uniform_initializer_create(int seed, float min, float max);
FF_RT_API void flexflow_uniform_initializer_destroy(flexflow_uniform_initializer_t handle);
FF_RT_API flexflow_norm_initializer_t flexflow_norm_initializer_create(int seed, float mean, float stddev);
FF_RT_API void flexflow_norm_initializer_destroy(flexflow_norm_initializer_t handle);

FF_RT_API void flexflow_per_metrics_destroy(flexflow_perf_metrics_t handle);
FF_RT_API float flexflow_per_metrics_get_accuracy(flexflow_perf_metrics_t handle);

/* ---- example configs (NetConfig, DLRMConfig) ---------------------------- */
FF_RT_API flexflow_net_config_t flexflow_net_config_create(void);
FF_RT_API void flexflow_net_config_destroy(flexflow_net_config_t handle);
FF_RT_API const char* flexflow_net_config_get_dataset_path(flexflow_net_config_t handle);
FF_RT_API flexflow_dlrm_config_t flexflow_dlrm_config_create(void);
FF_RT_API void flexflow_dlrm_config_destroy(flexflow_dlrm_config_t handle);
FF_RT_API const char* flexflow_dlrm_config_get_dataset_path(flexflow_dlrm_config_t handle);
FF_RT_API const char* flexflow_dlrm_config_get_arch_interaction_op(flexflow_dlrm_config_t handle);
FF_RT_API int flexflow_dlrm_config_get_sparse_feature_size(flexflow_dlrm_config_t handle);
FF_RT_API int flexflow_dlrm_config_get_sigmoid_bot(flexflow_dlrm_config_t handle);
FF_RT_API int flexflow_dlrm_config_get_sigmoid_top(flexflow_dlrm_config_t handle);
FF_RT_API int flexflow_dlrm_config_get_embedding_bag_size(flexflow_dlrm_config_t handle);
FF_RT_API float flexflow_dlrm_config_get_loss_threshold(flexflow_dlrm_config_t handle);
/* int arrays: element 0 is the count, the values follow */
FF_RT_API int* flexflow_dlrm_config_get_mlp_bot(flexflow_dlrm_config_t handle);
FF_RT_API int* flexflow_dlrm_config_get_mlp_top(flexflow_dlrm_config_t handle);
FF_RT_API int* flexflow_dlrm_config_get_embedding_size(flexflow_dlrm_config_t handle);

/* ---- SingleDataLoader: batches of a full-dataset tensor / host buffer --- */
FF_RT_API flexflow_single_dataloader_t flexflow_single_dataloader_create(flexflow_model_t ffmodel,
                                                                         flexflow_tensor_t input,
                                                                         flexflow_tensor_t full_input,
                                                                         int num_samples, enum DataType data_type);
FF_RT_API flexflow_single_dataloader_t flexflow_single_dataloader_create2(flexflow_model_t ffmodel,
                                                                          flexflow_tensor_t input,
                                                                          void* full_input_ptr, int num_samples,
                                                                          enum DataType data_type);
FF_RT_API void flexflow_single_dataloader_destroy(flexflow_single_dataloader_t handle);
FF_RT_API void flexflow_single_dataloader_set_num_samples(flexflow_single_dataloader_t handle, int samples);
FF_RT_API int flexflow_single_dataloader_get_num_samples(flexflow_single_dataloader_t handle);
FF_RT_API void flexflow_single_dataloader_reset(flexflow_single_dataloader_t handle);
/* the reference's spelling of next_batch is kept, and the correct one added */
FF_RT_API void flowflow_single_dataloader_next_batch(flexflow_single_dataloader_t handle, flexflow_model_t ffmodel);
FF_RT_API void flexflow_single_dataloader_next_batch(flexflow_single_dataloader_t handle, flexflow_model_t ffmodel);

/* ---- timing / tracing ---------------------------------------------------- */
FF_RT_API double flexflow_get_current_time(flexflow_config_t config);  /* microseconds */
FF_RT_API void flexflow_begin_trace(flexflow_config_t config, int trace_id);
FF_RT_API void flexflow_end_trace(flexflow_config_t config, int trace_id);

/* ---- Op ------------------------------------------------------------------ */
FF_RT_API int flexflow_op_get_num_parameters(flexflow_op_t handle);
FF_RT_API flexflow_tensor_t flexflow_op_get_parameter_by_id(flexflow_op_t handle, int id);
FF_RT_API int flexflow_op_get_num_inputs(flexflow_op_t handle);
FF_RT_API flexflow_tensor_t flexflow_op_get_input_by_id(flexflow_op_t handle, int id);
FF_RT_API int flexflow_op_get_num_outputs(flexflow_op_t handle);
FF_RT_API flexflow_tensor_t flexflow_op_get_output_by_id(flexflow_op_t handle, int id);
FF_RT_API void flexflow_op_init(flexflow_op_t handle, flexflow_model_t model);
FF_RT_API void flexflow_op_forward(flexflow_op_t handle, flexflow_model_t model);

/* ---- task entry points of the reference's Legion top-level task ---------- */
FF_RT_API void register_c_custom_tasks(void);
FF_RT_API void begin_flexflow_task(int argc, char** argv);
FF_RT_API void finish_flexflow_task(void);

#ifdef __cplusplus
}
#endif
#endif /* FLEXFLOW_RUNTIME_C_H */
