/* C ABI of the MI355X framework core (libflexflow_c.so).
 *
 * Parity: the reference's C FFI headers lib/pcg/ffi/include/flexflow/pcg.h
 * (computation-graph build + (de)serialisation, :41-360),
 * lib/compiler/ffi/include/flexflow/compiler.h (graph optimisation and its
 * search result, :24-34) and the op-attrs / utils error conventions.  The
 * handles are opaque pointers; tensors are plain value handles
 * {layer node, output index}.  Every call returns FLEXFLOW_OK (0) or an error
 * code; flexflow_last_error() returns the message of the calling thread's
 * last failure.  Strings returned through `char**` are malloc'd: release them
 * with flexflow_free().
 *
 * Training itself runs in the per-rank Python executor (one process per GPU
 * over RCCL); a C host drives it through the CLI / Python entry points, the
 * C ABI covers graph construction, serialisation and strategy search.
 */
#ifndef FLEXFLOW_C_H
#define FLEXFLOW_C_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FLEXFLOW_C_API __attribute__((visibility("default")))

typedef int flexflow_error_t;
enum {
  FLEXFLOW_OK = 0,
  FLEXFLOW_ERROR_INVALID_ARGUMENT = 1,
  FLEXFLOW_ERROR_SHAPE = 2,
  FLEXFLOW_ERROR_IO = 3,
  FLEXFLOW_ERROR_INTERNAL = 4,
};

typedef enum {
  FLEXFLOW_DT_BOOL = 0,
  FLEXFLOW_DT_INT32 = 1,
  FLEXFLOW_DT_INT64 = 2,
  FLEXFLOW_DT_HALF = 3,
  FLEXFLOW_DT_BF16 = 4,
  FLEXFLOW_DT_FLOAT = 5,
  FLEXFLOW_DT_DOUBLE = 6,
} flexflow_datatype_t;

typedef enum {
  FLEXFLOW_AC_NONE = 0,
  FLEXFLOW_AC_RELU = 1,
  FLEXFLOW_AC_SIGMOID = 2,
  FLEXFLOW_AC_TANH = 3,
  FLEXFLOW_AC_GELU = 4,
} flexflow_activation_t;

typedef struct flexflow_computation_graph_s* flexflow_computation_graph_t;
typedef struct flexflow_search_result_s* flexflow_search_result_t;
typedef struct {
  int node;
  int idx;
} flexflow_tensor_t;

FLEXFLOW_C_API const char* flexflow_last_error(void);
FLEXFLOW_C_API void flexflow_free(void* p);
FLEXFLOW_C_API const char* flexflow_version(void);

/* ---- computation graph (pcg.h) */
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_create(flexflow_computation_graph_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_destroy(flexflow_computation_graph_t cg);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_serialize_to_buf(flexflow_computation_graph_t cg,
                                                                            char** out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_deserialize_from_buf(const char* buf,
                                                                                flexflow_computation_graph_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_serialize_to_file(flexflow_computation_graph_t cg,
                                                                             const char* path);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_deserialize_from_file(const char* path,
                                                                                 flexflow_computation_graph_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_as_dot(flexflow_computation_graph_t cg, char** out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_num_layers(flexflow_computation_graph_t cg, int* out);
/* named built-in model: "bert", "transformer", "inception_v3", "candle_uno", "split_test", ... */
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_from_model(const char* name,
                                                                      flexflow_computation_graph_t* out);

/* ---- tensors */
FLEXFLOW_C_API flexflow_error_t flexflow_tensor_create(flexflow_computation_graph_t cg, int num_dims,
                                                       const int64_t* dims, flexflow_datatype_t dtype,
                                                       bool create_grad, const char* name,
                                                       flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_tensor_get_num_dims(flexflow_computation_graph_t cg, flexflow_tensor_t t,
                                                             int* out);
FLEXFLOW_C_API flexflow_error_t flexflow_tensor_get_dims(flexflow_computation_graph_t cg, flexflow_tensor_t t,
                                                         int64_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_tensor_get_datatype(flexflow_computation_graph_t cg, flexflow_tensor_t t,
                                                             flexflow_datatype_t* out);

/* ---- operators.  Generic form: `attrs_json` is an operator attribute
 * object {"op_type": "LINEAR", "out_channels": 64, ...}; outputs are written
 * to `outputs` (capacity `max_outputs`), their count to `num_outputs`. */
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op(flexflow_computation_graph_t cg,
                                                                  const char* attrs_json, int num_inputs,
                                                                  const flexflow_tensor_t* inputs, const char* name,
                                                                  int max_outputs, flexflow_tensor_t* outputs,
                                                                  int* num_outputs);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_dense(flexflow_computation_graph_t cg,
                                                                        flexflow_tensor_t x, int64_t out_dim,
                                                                        flexflow_activation_t act, bool use_bias,
                                                                        const char* name, flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_relu(flexflow_computation_graph_t cg,
                                                                       flexflow_tensor_t x, const char* name,
                                                                       flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_gelu(flexflow_computation_graph_t cg,
                                                                       flexflow_tensor_t x, const char* name,
                                                                       flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_sigmoid(flexflow_computation_graph_t cg,
                                                                          flexflow_tensor_t x, const char* name,
                                                                          flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_tanh(flexflow_computation_graph_t cg,
                                                                       flexflow_tensor_t x, const char* name,
                                                                       flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_exp(flexflow_computation_graph_t cg,
                                                                      flexflow_tensor_t x, const char* name,
                                                                      flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_identity(flexflow_computation_graph_t cg,
                                                                           flexflow_tensor_t x, const char* name,
                                                                           flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_rsqrt(flexflow_computation_graph_t cg,
                                                                        flexflow_tensor_t x, const char* name,
                                                                        flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_scalar_multiply(flexflow_computation_graph_t cg,
                                                                                  flexflow_tensor_t x, double s,
                                                                                  const char* name,
                                                                                  flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_scalar_add(flexflow_computation_graph_t cg,
                                                                             flexflow_tensor_t x, double s,
                                                                             const char* name, flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_add(flexflow_computation_graph_t cg,
                                                                      flexflow_tensor_t a, flexflow_tensor_t b,
                                                                      const char* name, flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_subtract(flexflow_computation_graph_t cg,
                                                                           flexflow_tensor_t a, flexflow_tensor_t b,
                                                                           const char* name, flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_multiply(flexflow_computation_graph_t cg,
                                                                           flexflow_tensor_t a, flexflow_tensor_t b,
                                                                           const char* name, flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_divide(flexflow_computation_graph_t cg,
                                                                         flexflow_tensor_t a, flexflow_tensor_t b,
                                                                         const char* name, flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_softmax(flexflow_computation_graph_t cg,
                                                                          flexflow_tensor_t x, int dim,
                                                                          const char* name, flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_layer_norm(flexflow_computation_graph_t cg,
                                                                             flexflow_tensor_t x, int num_axes,
                                                                             const int64_t* axes, bool affine,
                                                                             double eps, const char* name,
                                                                             flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_batch_norm(flexflow_computation_graph_t cg,
                                                                             flexflow_tensor_t x, bool relu,
                                                                             const char* name, flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_embedding(flexflow_computation_graph_t cg,
                                                                            flexflow_tensor_t x, int64_t num_entries,
                                                                            int64_t out_dim, const char* aggr,
                                                                            const char* name, flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_batch_matmul(flexflow_computation_graph_t cg,
                                                                               flexflow_tensor_t a, flexflow_tensor_t b,
                                                                               const char* name,
                                                                               flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_conv2d(
    flexflow_computation_graph_t cg, flexflow_tensor_t x, int64_t out_channels, int kernel_h, int kernel_w,
    int stride_h, int stride_w, int padding_h, int padding_w, flexflow_activation_t act, int groups, bool use_bias,
    const char* name, flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_pool2d(
    flexflow_computation_graph_t cg, flexflow_tensor_t x, int kernel_h, int kernel_w, int stride_h, int stride_w,
    int padding_h, int padding_w, const char* pool_type, const char* name, flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_flat(flexflow_computation_graph_t cg,
                                                                       flexflow_tensor_t x, const char* name,
                                                                       flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_reshape(flexflow_computation_graph_t cg,
                                                                          flexflow_tensor_t x, int num_dims,
                                                                          const int64_t* shape, const char* name,
                                                                          flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_transpose(flexflow_computation_graph_t cg,
                                                                            flexflow_tensor_t x, int num_dims,
                                                                            const int64_t* perm, const char* name,
                                                                            flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_concat(flexflow_computation_graph_t cg,
                                                                         int num_inputs, const flexflow_tensor_t* xs,
                                                                         int axis, const char* name,
                                                                         flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_split(flexflow_computation_graph_t cg,
                                                                        flexflow_tensor_t x, int num_splits,
                                                                        const int64_t* sizes, int axis,
                                                                        const char* name, flexflow_tensor_t* outs);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_op_dropout(flexflow_computation_graph_t cg,
                                                                          flexflow_tensor_t x, double rate,
                                                                          int64_t seed, const char* name,
                                                                          flexflow_tensor_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_add_multihead_attention(
    flexflow_computation_graph_t cg, flexflow_tensor_t q, flexflow_tensor_t k, flexflow_tensor_t v,
    int64_t embed_dim, int64_t num_heads, int64_t kdim, int64_t vdim, double dropout, bool bias, bool causal,
    const char* name, flexflow_tensor_t* out);

/* ---- compiler (compiler.h).  machine_json: MachineSpecification fields
 * ({"num_nodes":1,"num_gpus_per_node":8,...}; empty -> one MI355X node);
 * search_json: {"algorithm": "unity"|"mcmc"|"data_parallel", "world": 8,
 * "budget": ..., "alpha": ..., ...}. */
FLEXFLOW_C_API flexflow_error_t flexflow_computation_graph_optimize(flexflow_computation_graph_t cg,
                                                                    const char* machine_json,
                                                                    const char* search_json,
                                                                    flexflow_search_result_t* out);
FLEXFLOW_C_API flexflow_error_t flexflow_search_result_destroy(flexflow_search_result_t r);
FLEXFLOW_C_API flexflow_error_t flexflow_search_result_get_cost(flexflow_search_result_t r, double* seconds,
                                                                double* data_parallel_seconds);
/* the search report (strategy, cost trace, views) as JSON */
FLEXFLOW_C_API flexflow_error_t flexflow_search_result_get_report_json(flexflow_search_result_t r, char** out);
/* the parallel computation graph (JSON v1) */
FLEXFLOW_C_API flexflow_error_t flexflow_search_result_get_parallel_computation_graph_json(
    flexflow_search_result_t r, char** out);
/* PCG layer producing the parallel version of a CG tensor (-1 if none) */
FLEXFLOW_C_API flexflow_error_t flexflow_search_result_get_parallel_layer_for_layer(flexflow_search_result_t r,
                                                                                   int cg_node, int* pcg_node);

#ifdef __cplusplus
}
#endif
#endif /* FLEXFLOW_C_H */
