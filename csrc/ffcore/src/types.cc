#include "ff/types.h"

#include <sstream>
#include <unordered_map>

namespace ff {

size_t size_of(DataType dt) {
  switch (dt) {
    case DataType::BOOL: return 1;
    case DataType::INT32: return 4;
    case DataType::INT64: return 8;
    case DataType::HALF: return 2;
    case DataType::BFLOAT16: return 2;
    case DataType::FLOAT: return 4;
    case DataType::DOUBLE: return 8;
    case DataType::FP8_E4M3: return 1;
    case DataType::NONE: return 0;
  }
  return 0;
}

static const char* kDtNames[] = {"bool", "int32", "int64", "half", "bfloat16",
                                 "float", "double", "fp8_e4m3", "none"};

std::string to_string(DataType dt) { return kDtNames[static_cast<int>(dt)]; }

DataType datatype_from_string(const std::string& s) {
  for (int i = 0; i <= static_cast<int>(DataType::NONE); ++i)
    if (s == kDtNames[i]) return static_cast<DataType>(i);
  if (s == "float32" || s == "fp32") return DataType::FLOAT;
  if (s == "bf16") return DataType::BFLOAT16;
  if (s == "float16" || s == "fp16") return DataType::HALF;
  if (s == "float64") return DataType::DOUBLE;
  throw FFError("unknown datatype " + s);
}

static const char* kOpNames[] = {
#define FF_STR_ITEM(n) #n,
    FF_OP_TYPES(FF_STR_ITEM)
#undef FF_STR_ITEM
};

std::string to_string(OpType t) { return kOpNames[static_cast<int>(t)]; }

OpType optype_from_string(const std::string& s) {
  static std::unordered_map<std::string, OpType> m = [] {
    std::unordered_map<std::string, OpType> r;
    for (int i = 0; i < static_cast<int>(OpType::NUM_OP_TYPES); ++i)
      r[kOpNames[i]] = static_cast<OpType>(i);
    return r;
  }();
  auto it = m.find(s);
  if (it == m.end()) throw FFError("unknown operator type " + s);
  return it->second;
}

std::vector<OpType> all_op_types() {
  std::vector<OpType> r;
  for (int i = 0; i < static_cast<int>(OpType::NUM_OP_TYPES); ++i) r.push_back(static_cast<OpType>(i));
  return r;
}

bool is_parallel_op(OpType t) {
  return t == OpType::REPARTITION || t == OpType::COMBINE || t == OpType::REPLICATE ||
         t == OpType::REDUCTION || t == OpType::FUSED_PARALLEL || t == OpType::ALLTOALL ||
         t == OpType::PIPELINE;
}

bool is_elementwise_unary(OpType t) {
  switch (t) {
    case OpType::RELU: case OpType::SIGMOID: case OpType::TANH: case OpType::ELU:
    case OpType::GELU: case OpType::EXP: case OpType::LOG: case OpType::SQRT:
    case OpType::RSQRT: case OpType::SIN: case OpType::COS: case OpType::POW:
    case OpType::IDENTITY: case OpType::CEIL: case OpType::ROUND:
    case OpType::LOGICAL_NOT: case OpType::LEAKYRELU: case OpType::SCALAR_MULTIPLY:
    case OpType::SCALAR_ADD: case OpType::SCALAR_SUB: case OpType::SCALAR_TRUE_DIV:
    case OpType::SCALAR_FLOOR_DIV:
      return true;
    default: return false;
  }
}

bool is_elementwise_binary(OpType t) {
  switch (t) {
    case OpType::EW_ADD: case OpType::EW_SUB: case OpType::EW_MUL: case OpType::EW_DIV:
    case OpType::EW_MAX: case OpType::EW_MIN: case OpType::EW_EQUAL:
    case OpType::EW_GREATER: case OpType::EW_LESS:
      return true;
    default: return false;
  }
}

std::string to_string(Activation a) {
  switch (a) {
    case Activation::NONE: return "none";
    case Activation::RELU: return "relu";
    case Activation::SIGMOID: return "sigmoid";
    case Activation::TANH: return "tanh";
    case Activation::GELU: return "gelu";
  }
  return "none";
}

Activation activation_from_string(const std::string& s) {
  if (s == "none" || s.empty()) return Activation::NONE;
  if (s == "relu") return Activation::RELU;
  if (s == "sigmoid") return Activation::SIGMOID;
  if (s == "tanh") return Activation::TANH;
  if (s == "gelu") return Activation::GELU;
  throw FFError("unknown activation " + s);
}

// ---------------------------------------------------------------------------
int64_t TensorShape::at(int idx) const { return dims.at(normalize_dim(idx, num_dims())); }
int64_t& TensorShape::at(int idx) { return dims.at(normalize_dim(idx, num_dims())); }
int64_t TensorShape::num_elements() const { return product(dims); }

std::string TensorShape::str() const {
  std::ostringstream os;
  os << "[";
  for (size_t i = 0; i < dims.size(); ++i) os << (i ? ", " : "") << dims[i];
  os << "]:" << to_string(dtype);
  return os.str();
}

Json TensorShape::to_json() const {
  Json j = Json::object();
  j["dims"] = Json(dims);
  j["data_type"] = to_string(dtype);
  return j;
}

TensorShape TensorShape::from_json(const Json& j) {
  TensorShape s;
  s.dims = j.at("dims").as_int_vector();
  s.dtype = datatype_from_string(j.at("data_type").as_string());
  return s;
}

const ShardParallelDim& ParallelTensorShape::dim(int idx) const {
  return shard_dims.at(normalize_dim(idx, num_dims()));
}
ShardParallelDim& ParallelTensorShape::dim(int idx) {
  return shard_dims.at(normalize_dim(idx, num_dims()));
}

int ParallelTensorShape::total_parallel_degree() const {
  int r = sum_degree * discard_copy_degree;
  for (auto const& d : shard_dims) r *= d.degree;
  return r;
}

std::vector<int> ParallelTensorShape::shard_degrees() const {
  std::vector<int> r;
  for (auto const& d : shard_dims) r.push_back(d.degree);
  return r;
}

TensorShape ParallelTensorShape::reduced_shape() const {
  TensorShape s;
  s.dtype = dtype;
  for (auto const& d : shard_dims) s.dims.push_back(d.size);
  return s;
}

TensorShape ParallelTensorShape::piece_shape() const {
  TensorShape s;
  s.dtype = dtype;
  for (auto const& d : shard_dims) s.dims.push_back((d.size + d.degree - 1) / d.degree);
  return s;
}

bool ParallelTensorShape::is_valid() const {
  if (sum_degree < 1 || discard_copy_degree < 1) return false;
  for (auto const& d : shard_dims)
    if (d.degree < 1 || d.size % d.degree != 0) return false;
  return true;
}

bool ParallelTensorShape::operator<(const ParallelTensorShape& o) const {
  if (shard_dims != o.shard_dims) return shard_dims < o.shard_dims;
  if (sum_degree != o.sum_degree) return sum_degree < o.sum_degree;
  if (discard_copy_degree != o.discard_copy_degree) return discard_copy_degree < o.discard_copy_degree;
  return dtype < o.dtype;
}

std::string ParallelTensorShape::str() const {
  std::ostringstream os;
  os << "[";
  for (size_t i = 0; i < shard_dims.size(); ++i)
    os << (i ? ", " : "") << shard_dims[i].size << "/" << shard_dims[i].degree;
  os << "] sum=" << sum_degree << " copy=" << discard_copy_degree << " " << to_string(dtype);
  return os.str();
}

Json ParallelTensorShape::to_json() const {
  Json j = Json::object();
  Json dims = Json::array();
  for (auto const& d : shard_dims) {
    Json e = Json::object();
    e["size"] = d.size;
    e["degree"] = d.degree;
    dims.push_back(e);
  }
  j["shard_dims"] = dims;
  j["sum_degree"] = sum_degree;
  j["discard_copy_degree"] = discard_copy_degree;
  j["data_type"] = to_string(dtype);
  return j;
}

ParallelTensorShape ParallelTensorShape::from_json(const Json& j) {
  ParallelTensorShape s;
  for (auto const& e : j.at("shard_dims").as_array())
    s.shard_dims.push_back({e.at("size").as_int(), static_cast<int>(e.at("degree").as_int())});
  s.sum_degree = static_cast<int>(j.at("sum_degree").as_int());
  s.discard_copy_degree = static_cast<int>(j.at("discard_copy_degree").as_int());
  s.dtype = datatype_from_string(j.at("data_type").as_string());
  return s;
}

ParallelTensorShape lift_to_parallel(const TensorShape& s) {
  ParallelTensorShape p;
  p.dtype = s.dtype;
  for (auto d : s.dims) p.shard_dims.push_back({d, 1});
  return p;
}

ParallelTensorShape lift_to_parallel_with_degrees(const TensorShape& s, int sum_degree,
                                                  int discard_copy_degree,
                                                  const std::vector<int>& shard_degrees) {
  if (shard_degrees.size() != s.dims.size())
    throw FFError("lift_to_parallel_with_degrees: rank mismatch");
  ParallelTensorShape p = lift_to_parallel(s);
  for (size_t i = 0; i < shard_degrees.size(); ++i) p.shard_dims[i].degree = shard_degrees[i];
  p.sum_degree = sum_degree;
  p.discard_copy_degree = discard_copy_degree;
  return p;
}

}  // namespace ff
