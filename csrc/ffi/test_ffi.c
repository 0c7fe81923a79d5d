/* Exercises the C ABI end to end: build an MLP, (de)serialise it, run the
 * strategy search for 8 GPUs, query the result.  Prints "FFI OK". */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "flexflow_c.h"

#define CHECK(x)                                                             \
  do {                                                                       \
    flexflow_error_t e_ = (x);                                               \
    if (e_ != FLEXFLOW_OK) {                                                 \
      fprintf(stderr, "%s failed (%d): %s\n", #x, e_, flexflow_last_error()); \
      return 1;                                                              \
    }                                                                        \
  } while (0)

int main(int argc, char** argv) {
  const char* tmp = argc > 1 ? argv[1] : "/tmp/ffi_cg.json";
  flexflow_computation_graph_t cg;
  CHECK(flexflow_computation_graph_create(&cg));
  int64_t dims[2] = {64, 256};
  flexflow_tensor_t x, h, y, z;
  CHECK(flexflow_tensor_create(cg, 2, dims, FLEXFLOW_DT_FLOAT, true, "x", &x));
  CHECK(flexflow_computation_graph_add_op_dense(cg, x, 512, FLEXFLOW_AC_RELU, true, "fc1", &h));
  CHECK(flexflow_computation_graph_add_op_dense(cg, h, 256, FLEXFLOW_AC_NONE, true, "fc2", &y));
  CHECK(flexflow_computation_graph_add_op_add(cg, x, y, "res", &z));
  flexflow_tensor_t g[1];
  int n = 0;
  CHECK(flexflow_computation_graph_add_op(cg, "{\"op_type\": \"SOFTMAX\", \"dim\": -1}", 1, &z, "sm", 1, g, &n));
  if (n != 1) return 2;
  int64_t od[2];
  int nd = 0;
  CHECK(flexflow_tensor_get_num_dims(cg, g[0], &nd));
  CHECK(flexflow_tensor_get_dims(cg, g[0], od));
  if (nd != 2 || od[0] != 64 || od[1] != 256) return 3;
  /* a shape error is reported, not thrown */
  flexflow_tensor_t bad;
  int64_t d3[1] = {7};
  flexflow_tensor_t w;
  CHECK(flexflow_tensor_create(cg, 1, d3, FLEXFLOW_DT_FLOAT, true, "w", &w));
  if (flexflow_computation_graph_add_op_add(cg, x, w, "bad", &bad) == FLEXFLOW_OK) return 4;
  if (strlen(flexflow_last_error()) == 0) return 5;

  CHECK(flexflow_computation_graph_serialize_to_file(cg, tmp));
  flexflow_computation_graph_t cg2;
  CHECK(flexflow_computation_graph_deserialize_from_file(tmp, &cg2));
  int l1 = 0, l2 = 0;
  CHECK(flexflow_computation_graph_num_layers(cg, &l1));
  CHECK(flexflow_computation_graph_num_layers(cg2, &l2));
  if (l1 != l2) return 6;

  flexflow_search_result_t r;
  CHECK(flexflow_computation_graph_optimize(cg2, "{\"num_nodes\":1,\"num_gpus_per_node\":8}",
                                            "{\"algorithm\":\"mcmc\",\"budget\":50,\"seed\":1}", &r));
  double c = 0, dp = 0;
  CHECK(flexflow_search_result_get_cost(r, &c, &dp));
  if (!(c > 0 && dp > 0 && c <= dp * 1.0001)) return 7;
  char* pcg = NULL;
  CHECK(flexflow_search_result_get_parallel_computation_graph_json(r, &pcg));
  if (!pcg || strlen(pcg) < 10) return 8;
  flexflow_free(pcg);
  char* rep = NULL;
  CHECK(flexflow_search_result_get_report_json(r, &rep));
  flexflow_free(rep);
  int pn = -1;
  CHECK(flexflow_search_result_get_parallel_layer_for_layer(r, h.node, &pn));
  if (pn < 0) return 9;
  CHECK(flexflow_search_result_destroy(r));

  flexflow_computation_graph_t bert;
  CHECK(flexflow_computation_graph_from_model("bert", &bert));
  int lb = 0;
  CHECK(flexflow_computation_graph_num_layers(bert, &lb));
  if (lb < 10) return 10;
  CHECK(flexflow_computation_graph_destroy(bert));
  CHECK(flexflow_computation_graph_destroy(cg2));
  CHECK(flexflow_computation_graph_destroy(cg));
  printf("FFI OK layers=%d cost=%.6g dp=%.6g %s\n", l1, c, dp, flexflow_version());
  return 0;
}
