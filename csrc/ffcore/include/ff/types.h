// Core IR value types: datatypes, operator kinds, tensor shapes and parallel
// tensor shapes.
//
// Parity:
//  * OperatorType vocabulary: lib/op-attrs/include/op-attrs/operator_type.enum.toml:10-94
//  * DataType: lib/op-attrs/include/op-attrs/datatype.enum.toml (+ bf16/fp8 for CDNA4)
//  * ParallelTensorShape {shard dims (size, degree), sum_degree, discard_copy_degree}:
//    lib/op-attrs/include/op-attrs/parallel_tensor_shape.struct.toml,
//    parallel_tensor_dims.struct.toml, replica_parallel_dim_set.struct.toml,
//    lib/op-attrs/src/op-attrs/parallel_tensor_shape.cc:13-146
//
// Dims are row-major, dims[0] is the outermost (sample) dimension, negative
// indices count from the innermost dimension (the reference's FFOrdered /
// ff_dim_t{-1} convention).
#pragma once
#include <cstdint>
#include <functional>
#include <optional>
#include <string>
#include <vector>

#include "ff/json.h"

namespace ff {

enum class DataType : int {
  BOOL = 0,
  INT32,
  INT64,
  HALF,
  BFLOAT16,
  FLOAT,
  DOUBLE,
  FP8_E4M3,
  NONE,
};
size_t size_of(DataType dt);
std::string to_string(DataType dt);
DataType datatype_from_string(const std::string& s);

#define FF_OP_TYPES(X)                                                          \
  X(NOOP) X(INPUT) X(WEIGHT) X(CONV2D) X(DROPOUT) X(LINEAR) X(BATCHMATMUL)      \
  X(POOL2D) X(SCALAR_MULTIPLY) X(SCALAR_ADD) X(SCALAR_FLOOR_DIV)               \
  X(SCALAR_TRUE_DIV) X(SCALAR_SUB) X(RELU) X(IDENTITY) X(SIGMOID) X(TANH)      \
  X(ELU) X(FLAT) X(SOFTMAX) X(BATCHNORM) X(CONCAT) X(SPLIT) X(EMBEDDING)       \
  X(CACHE) X(RESHAPE) X(REVERSE) X(TRANSPOSE) X(EW_ADD) X(EW_MUL) X(MATMUL)    \
  X(MUL) X(ENLARGE) X(SQUEEZE) X(UNSQUEEZE) X(EW_SUB) X(EW_DIV) X(EW_EQUAL)    \
  X(EW_GREATER) X(EW_LESS) X(EW_MAX) X(EW_MIN) X(REDUCE_ARGMAX)                \
  X(REDUCE_ARGMIN) X(REDUCE_MAX) X(REDUCE_MEAN) X(REDUCE_MIN) X(REDUCE_PROD)   \
  X(REDUCE_SUM) X(PAD) X(SHAPE) X(SIZE) X(TOPK) X(WHERE) X(CEIL) X(CAST)       \
  X(EXP) X(ROUND) X(LOG) X(LOGICAL_NOT) X(SQRT) X(SIN) X(COS) X(LEAKYRELU)     \
  X(SLICE) X(RESIZE) X(PRELU) X(GELU) X(MULTIHEAD_ATTENTION) X(FUSED) X(RSQRT) \
  X(POW) X(MEAN) X(LAYERNORM) X(GATHER) X(BROADCAST) X(REPARTITION) X(COMBINE) \
  X(REPLICATE) X(REDUCTION) X(BATCH) X(PIPELINE) X(FUSED_PARALLEL)             \
  X(ALLTOALL) X(EXPERTS)

enum class OpType : int {
#define FF_ENUM_ITEM(n) n,
  FF_OP_TYPES(FF_ENUM_ITEM)
#undef FF_ENUM_ITEM
      NUM_OP_TYPES
};
std::string to_string(OpType t);
OpType optype_from_string(const std::string& s);
std::vector<OpType> all_op_types();
bool is_parallel_op(OpType t);
bool is_elementwise_unary(OpType t);
bool is_elementwise_binary(OpType t);

enum class Activation : int { NONE = 0, RELU, SIGMOID, TANH, GELU };
std::string to_string(Activation a);
Activation activation_from_string(const std::string& s);

enum class AggrMode : int { NONE = 0, SUM, AVG };
enum class PoolType : int { MAX = 0, AVG };

// ---------------------------------------------------------------------------
// Serial shapes
struct TensorShape {
  std::vector<int64_t> dims;
  DataType dtype = DataType::FLOAT;

  int num_dims() const { return static_cast<int>(dims.size()); }
  int64_t at(int idx) const;  // negative index from the end
  int64_t& at(int idx);
  int64_t num_elements() const;
  int64_t size_bytes() const { return num_elements() * static_cast<int64_t>(size_of(dtype)); }
  bool operator==(const TensorShape& o) const { return dims == o.dims && dtype == o.dtype; }
  bool operator!=(const TensorShape& o) const { return !(*this == o); }
  bool operator<(const TensorShape& o) const {
    return dims != o.dims ? dims < o.dims : dtype < o.dtype;
  }
  std::string str() const;
  Json to_json() const;
  static TensorShape from_json(const Json& j);
};

// ---------------------------------------------------------------------------
// Parallel shapes
struct ShardParallelDim {
  int64_t size = 1;
  int degree = 1;
  bool operator==(const ShardParallelDim& o) const { return size == o.size && degree == o.degree; }
  bool operator<(const ShardParallelDim& o) const {
    return size != o.size ? size < o.size : degree < o.degree;
  }
};

struct ParallelTensorShape {
  std::vector<ShardParallelDim> shard_dims;
  int sum_degree = 1;           // # partial-sum replicas (a Reduction is pending)
  int discard_copy_degree = 1;  // # identical replicas
  DataType dtype = DataType::FLOAT;

  int num_dims() const { return static_cast<int>(shard_dims.size()); }
  const ShardParallelDim& dim(int idx) const;
  ShardParallelDim& dim(int idx);
  // product(shard degrees) * sum * discard_copy
  int total_parallel_degree() const;
  std::vector<int> shard_degrees() const;
  // The logical (unpartitioned) shape.
  TensorShape reduced_shape() const;
  // The per-device piece.
  TensorShape piece_shape() const;
  bool is_valid() const;  // every degree divides its dim size
  bool operator==(const ParallelTensorShape& o) const {
    return shard_dims == o.shard_dims && sum_degree == o.sum_degree &&
           discard_copy_degree == o.discard_copy_degree && dtype == o.dtype;
  }
  bool operator!=(const ParallelTensorShape& o) const { return !(*this == o); }
  bool operator<(const ParallelTensorShape& o) const;
  std::string str() const;
  Json to_json() const;
  static ParallelTensorShape from_json(const Json& j);
};

// Lift a serial shape to a parallel shape with all degrees 1.
ParallelTensorShape lift_to_parallel(const TensorShape& s);
ParallelTensorShape lift_to_parallel_with_degrees(const TensorShape& s, int sum_degree,
                                                  int discard_copy_degree,
                                                  const std::vector<int>& shard_degrees);

struct FFError : public std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline int normalize_dim(int idx, int ndims) {
  int r = idx < 0 ? idx + ndims : idx;
  if (r < 0 || r >= ndims)
    throw FFError("dimension index " + std::to_string(idx) + " out of range for rank " +
                  std::to_string(ndims));
  return r;
}

template <typename T>
inline int64_t product(const std::vector<T>& xs) {
  int64_t r = 1;
  for (auto x : xs) r *= static_cast<int64_t>(x);
  return r;
}

inline size_t hash_combine(size_t seed, size_t v) {
  return seed ^ (v + 0x9e3779b97f4a7c15ULL + (seed << 6) + (seed >> 2));
}

}  // namespace ff

namespace std {
template <>
struct hash<ff::TensorShape> {
  size_t operator()(const ff::TensorShape& s) const {
    size_t h = std::hash<int>()(static_cast<int>(s.dtype));
    for (auto d : s.dims) h = ff::hash_combine(h, std::hash<int64_t>()(d));
    return h;
  }
};
template <>
struct hash<ff::ParallelTensorShape> {
  size_t operator()(const ff::ParallelTensorShape& s) const {
    size_t h = std::hash<int>()(static_cast<int>(s.dtype));
    for (auto d : s.shard_dims) {
      h = ff::hash_combine(h, std::hash<int64_t>()(d.size));
      h = ff::hash_combine(h, std::hash<int>()(d.degree));
    }
    h = ff::hash_combine(h, std::hash<int>()(s.sum_degree));
    h = ff::hash_combine(h, std::hash<int>()(s.discard_copy_degree));
    return h;
  }
};
}  // namespace std
