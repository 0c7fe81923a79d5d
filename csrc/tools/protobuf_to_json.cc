// ffc-protobuf-to-json: convert a TASO rule corpus in protobuf wire format
// (GraphSubst.RuleCollection, bin/protobuf_to_json/rules.proto) to the JSON
// corpus format (substitutions/graph_subst_3_v2.json).
//
// Parity: bin/protobuf_to_json/protobuf_to_json.cc (242 LoC; libprotobuf +
// nlohmann). No protobuf runtime is needed here: the schema is five flat
// messages of int32 fields, decoded straight from the wire format.
#include <cstdint>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "ff/json.h"

using ff::Json;

namespace {

const char* kOpTypes[] = {"OP_INPUT",        "OP_WEIGHT",         "OP_ANY",           "OP_CONV2D",
                          "OP_DROPOUT",      "OP_LINEAR",         "OP_POOL2D_MAX",    "OP_POOL2D_AVG",
                          "OP_RELU",         "OP_SIGMOID",        "OP_TANH",          "OP_BATCHNORM",
                          "OP_CONCAT",       "OP_SPLIT",          "OP_RESHAPE",       "OP_TRANSPOSE",
                          "OP_EW_ADD",       "OP_EW_MUL",         "OP_MATMUL",        "OP_MUL",
                          "OP_ENLARGE",      "OP_MERGE_GCONV",    "OP_CONSTANT_IMM",  "OP_CONSTANT_ICONV",
                          "OP_CONSTANT_ONE", "OP_CONSTANT_POOL",  "OP_PARTITION",     "OP_COMBINE",
                          "OP_REPLICATE",    "OP_REDUCE",         "OP_EMBEDDING"};
const char* kParams[] = {"PM_OP_TYPE",  "PM_NUM_INPUTS", "PM_NUM_OUTPUTS", "PM_GROUP",     "PM_KERNEL_H",
                         "PM_KERNEL_W", "PM_STRIDE_H",   "PM_STRIDE_W",    "PM_PAD",       "PM_ACTI",
                         "PM_NUMDIM",   "PM_AXIS",       "PM_PERM",        "PM_OUTSHUFFLE", "PM_MERGE_GCONV_COUNT",
                         "PM_PARALLEL_DIM", "PM_PARALLEL_DEGREE"};

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool done() const { return p >= end; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= end) throw std::runtime_error("truncated varint");
      uint8_t b = *p++;
      v |= uint64_t(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    throw std::runtime_error("bad varint");
  }
  // returns field number, sets wire type
  int tag(int& wt) {
    uint64_t t = varint();
    wt = static_cast<int>(t & 7);
    return static_cast<int>(t >> 3);
  }
  Reader sub() {
    uint64_t n = varint();
    if (p + n > end) throw std::runtime_error("truncated message");
    Reader r{p, p + n};
    p += n;
    return r;
  }
  void skip(int wt) {
    if (wt == 0) varint();
    else if (wt == 1) p += 8;
    else if (wt == 2) sub();
    else if (wt == 5) p += 4;
    else throw std::runtime_error("unsupported wire type");
  }
};

int32_t as_i32(uint64_t v) { return static_cast<int32_t>(static_cast<uint32_t>(v)); }

Json tensor(Reader r) {
  Json j = Json::object();
  j["_t"] = "Tensor";
  while (!r.done()) {
    int wt, f = r.tag(wt);
    if (f == 1 && wt == 0) j["opId"] = as_i32(r.varint());
    else if (f == 2 && wt == 0) j["tsId"] = as_i32(r.varint());
    else r.skip(wt);
  }
  return j;
}

Json parameter(Reader r) {
  Json j = Json::object();
  j["_t"] = "Parameter";
  while (!r.done()) {
    int wt, f = r.tag(wt);
    if (f == 1 && wt == 0) {
      int k = as_i32(r.varint());
      j["key"] = (k >= 0 && k < int(sizeof(kParams) / sizeof(*kParams))) ? Json(kParams[k]) : Json(k);
    } else if (f == 2 && wt == 0) {
      j["value"] = as_i32(r.varint());
    } else {
      r.skip(wt);
    }
  }
  return j;
}

Json op(Reader r) {
  Json j = Json::object();
  j["_t"] = "Operator";
  Json in = Json::array(), para = Json::array();
  while (!r.done()) {
    int wt, f = r.tag(wt);
    if (f == 1 && wt == 0) {
      int t = as_i32(r.varint());
      j["type"] = (t >= 0 && t < int(sizeof(kOpTypes) / sizeof(*kOpTypes))) ? Json(kOpTypes[t]) : Json(t);
    } else if (f == 2 && wt == 2) {
      in.push_back(tensor(r.sub()));
    } else if (f == 3 && wt == 2) {
      para.push_back(parameter(r.sub()));
    } else {
      r.skip(wt);
    }
  }
  j["input"] = in;
  j["para"] = para;
  return j;
}

Json map_output(Reader r) {
  Json j = Json::object();
  j["_t"] = "MapOutput";
  const char* names[] = {"", "srcOpId", "dstOpId", "srcTsId", "dstTsId"};
  while (!r.done()) {
    int wt, f = r.tag(wt);
    if (f >= 1 && f <= 4 && wt == 0) j[names[f]] = as_i32(r.varint());
    else r.skip(wt);
  }
  return j;
}

Json rule(Reader r, int idx) {
  Json j = Json::object();
  j["_t"] = "Rule";
  Json src = Json::array(), dst = Json::array(), mo = Json::array();
  while (!r.done()) {
    int wt, f = r.tag(wt);
    if (f == 1 && wt == 2) src.push_back(op(r.sub()));
    else if (f == 2 && wt == 2) dst.push_back(op(r.sub()));
    else if (f == 3 && wt == 2) mo.push_back(map_output(r.sub()));
    else r.skip(wt);
  }
  j["srcOp"] = src;
  j["dstOp"] = dst;
  j["mappedOutput"] = mo;
  j["name"] = "taso_rule_" + std::to_string(idx);
  return j;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 3) {
    std::cerr << "usage: ffc-protobuf-to-json RULES.pb OUT.json\n";
    return 2;
  }
  std::ifstream f(argv[1], std::ios::binary);
  if (!f) {
    std::cerr << "error: cannot open " << argv[1] << "\n";
    return 1;
  }
  std::string buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  try {
    Reader r{reinterpret_cast<const uint8_t*>(buf.data()), reinterpret_cast<const uint8_t*>(buf.data()) + buf.size()};
    Json rules = Json::array();
    int idx = 0;
    while (!r.done()) {
      int wt, fld = r.tag(wt);
      if (fld == 1 && wt == 2) rules.push_back(rule(r.sub(), idx++));
      else r.skip(wt);
    }
    Json out = Json::object();
    out["_t"] = "RuleCollection";
    out["rule"] = rules;
    std::ofstream o(argv[2]);
    o << out.dump(2) << "\n";
    std::cerr << "converted " << idx << " rules\n";
  } catch (const std::exception& e) {
    std::cerr << "error: " << e.what() << "\n";
    return 1;
  }
  return 0;
}
