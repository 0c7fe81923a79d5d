#include "ff/models.h"

#include <set>
#include <sstream>

namespace ff {

namespace {

std::string trunc_normal(double stddev) {
  std::ostringstream os;
  os << R"({"type":"truncated_normal","seed":0,"mean":0.0,"stddev":)" << stddev << R"(,"min_cutoff":)"
     << -2 * stddev << R"(,"max_cutoff":)" << 2 * stddev << "}";
  return os.str();
}
const char* kZero = R"({"type":"zero"})";
const char* kGlorotNormal = R"({"type":"glorot_normal","seed":0})";

template <typename T>
void get(const Json& j, const char* k, T& v) {
  if (!j.is_object() || !j.contains(k)) return;
  if constexpr (std::is_same_v<T, int64_t>) v = j.at(k).as_int();
  else if constexpr (std::is_same_v<T, double>) v = j.at(k).as_double();
  else if constexpr (std::is_same_v<T, bool>) v = j.at(k).as_bool();
  else if constexpr (std::is_same_v<T, std::string>) v = j.at(k).as_string();
}

}  // namespace

// ---------------------------------------------------------------------------
BertModelConfig BertModelConfig::from_json(const Json& j) {
  BertModelConfig c;
  get(j, "vocab_size", c.vocab_size);
  get(j, "hidden_size", c.hidden_size);
  get(j, "num_encoder_layers", c.num_encoder_layers);
  get(j, "num_heads", c.num_heads);
  get(j, "dim_feedforward", c.dim_feedforward);
  get(j, "sequence_length", c.sequence_length);
  get(j, "batch_size", c.batch_size);
  get(j, "hidden_act", c.hidden_act);
  get(j, "hidden_dropout_prob", c.hidden_dropout_prob);
  get(j, "attention_probs_dropout_prob", c.attention_probs_dropout_prob);
  get(j, "initializer_range", c.initializer_range);
  get(j, "layer_norm_eps", c.layer_norm_eps);
  get(j, "causal", c.causal);
  return c;
}

Json BertModelConfig::to_json() const {
  Json j = Json::object();
  j["vocab_size"] = vocab_size;
  j["hidden_size"] = hidden_size;
  j["num_encoder_layers"] = num_encoder_layers;
  j["num_heads"] = num_heads;
  j["dim_feedforward"] = dim_feedforward;
  j["sequence_length"] = sequence_length;
  j["batch_size"] = batch_size;
  j["hidden_act"] = hidden_act;
  j["hidden_dropout_prob"] = hidden_dropout_prob;
  j["attention_probs_dropout_prob"] = attention_probs_dropout_prob;
  j["initializer_range"] = initializer_range;
  j["layer_norm_eps"] = layer_norm_eps;
  j["causal"] = causal;
  return j;
}

ComputationGraph get_bert_computation_graph(const BertModelConfig& c) {
  ComputationGraph cg;
  const std::string proj = trunc_normal(c.initializer_range);
  Activation act = activation_from_string(c.hidden_act);
  ValueRef x = cg.create_input(TensorShape{{c.batch_size, c.sequence_length, c.hidden_size}, DataType::FLOAT},
                               true, "input");
  for (int64_t l = 0; l < c.num_encoder_layers; ++l) {
    std::string p = "layer" + std::to_string(l) + ".";
    ValueRef a = cg.multihead_attention(x, x, x, c.hidden_size, c.num_heads, 0, 0, c.attention_probs_dropout_prob,
                                        true, c.causal, p + "attention");
    ValueRef n = cg.layer_norm(cg.binary(OpType::EW_ADD, a, x, p + "attn_residual"), {-1}, true, c.layer_norm_eps,
                               p + "attn_ln");
    ValueRef h = cg.dense(n, c.dim_feedforward, act, true, p + "ffn1", proj, kZero);
    if (c.hidden_dropout_prob > 0) h = cg.dropout(h, c.hidden_dropout_prob, 0, p + "ffn1_dropout");
    h = cg.dense(h, c.hidden_size, Activation::NONE, true, p + "ffn2", proj, kZero);
    if (c.hidden_dropout_prob > 0) h = cg.dropout(h, c.hidden_dropout_prob, 0, p + "ffn2_dropout");
    x = cg.layer_norm(cg.binary(OpType::EW_ADD, n, h, p + "ffn_residual"), {-1}, true, c.layer_norm_eps,
                      p + "ffn_ln");
  }
  ValueRef logits = cg.dense(x, c.vocab_size, act, true, "decoder", proj, kZero);
  cg.softmax(logits, -1, "softmax");
  return cg;
}

// ---------------------------------------------------------------------------
TransformerModelConfig TransformerModelConfig::from_json(const Json& j) {
  TransformerModelConfig c;
  get(j, "num_features", c.num_features);
  get(j, "sequence_length", c.sequence_length);
  get(j, "batch_size", c.batch_size);
  get(j, "dim_feedforward", c.dim_feedforward);
  get(j, "num_heads", c.num_heads);
  get(j, "num_encoder_layers", c.num_encoder_layers);
  get(j, "num_decoder_layers", c.num_decoder_layers);
  get(j, "vocab_size", c.vocab_size);
  get(j, "dropout", c.dropout);
  get(j, "layer_norm_eps", c.layer_norm_eps);
  return c;
}

Json TransformerModelConfig::to_json() const {
  Json j = Json::object();
  j["num_features"] = num_features;
  j["sequence_length"] = sequence_length;
  j["batch_size"] = batch_size;
  j["dim_feedforward"] = dim_feedforward;
  j["num_heads"] = num_heads;
  j["num_encoder_layers"] = num_encoder_layers;
  j["num_decoder_layers"] = num_decoder_layers;
  j["vocab_size"] = vocab_size;
  j["dropout"] = dropout;
  j["layer_norm_eps"] = layer_norm_eps;
  return j;
}

ComputationGraph get_transformer_computation_graph(const TransformerModelConfig& c) {
  ComputationGraph cg;
  TensorShape s{{c.batch_size, c.sequence_length, c.num_features}, DataType::FLOAT};
  ValueRef input = cg.create_input(s, true, "input");
  ValueRef target = cg.create_input(s, true, "target");
  auto ffn = [&](ValueRef x, const std::string& p) {
    ValueRef h = cg.dense(x, c.dim_feedforward, Activation::RELU, true, p + "ffn1");
    if (c.dropout > 0) h = cg.dropout(h, c.dropout, 0, p + "ffn1_dropout");
    h = cg.dense(h, c.num_features, Activation::NONE, true, p + "ffn2");
    if (c.dropout > 0) h = cg.dropout(h, c.dropout, 0, p + "ffn2_dropout");
    return h;
  };
  auto ln = [&](ValueRef a, ValueRef b, const std::string& nm) {
    return cg.layer_norm(cg.binary(OpType::EW_ADD, a, b, nm + "_add"), {-1}, true, c.layer_norm_eps, nm);
  };
  ValueRef enc = input;
  for (int64_t l = 0; l < c.num_encoder_layers; ++l) {
    std::string p = "encoder" + std::to_string(l) + ".";
    ValueRef a = cg.multihead_attention(enc, enc, enc, c.num_features, c.num_heads, 0, 0, c.dropout, false, false,
                                        p + "self_attn");
    ValueRef n = ln(a, enc, p + "ln1");
    enc = ln(n, ffn(n, p), p + "ln2");
  }
  ValueRef dec = target;
  for (int64_t l = 0; l < c.num_decoder_layers; ++l) {
    std::string p = "decoder" + std::to_string(l) + ".";
    ValueRef a = cg.multihead_attention(dec, dec, dec, c.num_features, c.num_heads, 0, 0, c.dropout, false, false,
                                        p + "self_attn");
    ValueRef n1 = ln(dec, a, p + "ln1");
    ValueRef m = cg.multihead_attention(n1, enc, enc, c.num_features, c.num_heads, 0, 0, c.dropout, false, false,
                                        p + "cross_attn");
    ValueRef n2 = ln(n1, m, p + "ln2");
    dec = ln(n2, ffn(n2, p), p + "ln3");
  }
  cg.softmax(cg.dense(dec, c.vocab_size, Activation::RELU, true, "out_proj"), -1, "softmax");
  return cg;
}

// ---------------------------------------------------------------------------
InceptionV3ModelConfig InceptionV3ModelConfig::from_json(const Json& j) {
  InceptionV3ModelConfig c;
  get(j, "num_classes", c.num_classes);
  get(j, "batch_size", c.batch_size);
  get(j, "aux_logits", c.aux_logits);
  return c;
}

Json InceptionV3ModelConfig::to_json() const {
  Json j = Json::object();
  j["num_classes"] = num_classes;
  j["batch_size"] = batch_size;
  j["aux_logits"] = aux_logits;
  return j;
}

namespace {
struct Inception {
  ComputationGraph& cg;
  int n = 0;
  ValueRef conv(ValueRef x, int64_t oc, int kh, int kw, int sh = 1, int sw = 1, int ph = 0, int pw = 0) {
    std::string p = "conv" + std::to_string(n++);
    ValueRef t = cg.conv2d(x, oc, kh, kw, sh, sw, ph, pw, Activation::NONE, 1, false, p);
    return cg.batch_norm(t, true, p + "_bn");
  }
  ValueRef avg(ValueRef x) { return cg.pool2d(x, 3, 3, 1, 1, 1, 1, "avg", Activation::NONE, "pool" + std::to_string(n++)); }
  ValueRef maxp(ValueRef x) { return cg.pool2d(x, 3, 3, 2, 2, 0, 0, "max", Activation::NONE, "pool" + std::to_string(n++)); }
  ValueRef cat(const std::vector<ValueRef>& xs) { return cg.concat(xs, 1, "mixed" + std::to_string(n++)); }

  ValueRef a(ValueRef x, int64_t pool_features) {
    ValueRef b1 = conv(x, 64, 1, 1);
    ValueRef b5 = conv(conv(x, 48, 1, 1), 64, 5, 5, 1, 1, 2, 2);
    ValueRef b3 = conv(conv(conv(x, 64, 1, 1), 96, 3, 3, 1, 1, 1, 1), 96, 3, 3, 1, 1, 1, 1);
    ValueRef bp = conv(avg(x), pool_features, 1, 1);
    return cat({b1, b5, b3, bp});
  }
  ValueRef b(ValueRef x) {
    ValueRef b3 = conv(x, 384, 3, 3, 2, 2);
    ValueRef bd = conv(conv(conv(x, 64, 1, 1), 96, 3, 3, 1, 1, 1, 1), 96, 3, 3, 2, 2);
    return cat({b3, bd, maxp(x)});
  }
  ValueRef c(ValueRef x, int64_t c7) {
    ValueRef b1 = conv(x, 192, 1, 1);
    ValueRef b7 = conv(conv(conv(x, c7, 1, 1), c7, 1, 7, 1, 1, 0, 3), 192, 7, 1, 1, 1, 3, 0);
    ValueRef bd = conv(x, c7, 1, 1);
    bd = conv(bd, c7, 7, 1, 1, 1, 3, 0);
    bd = conv(bd, c7, 1, 7, 1, 1, 0, 3);
    bd = conv(bd, c7, 7, 1, 1, 1, 3, 0);
    bd = conv(bd, 192, 1, 7, 1, 1, 0, 3);
    ValueRef bp = conv(avg(x), 192, 1, 1);
    return cat({b1, b7, bd, bp});
  }
  ValueRef d(ValueRef x) {
    ValueRef b3 = conv(conv(x, 192, 1, 1), 320, 3, 3, 2, 2);
    ValueRef b7 = conv(x, 192, 1, 1);
    b7 = conv(b7, 192, 1, 7, 1, 1, 0, 3);
    b7 = conv(b7, 192, 7, 1, 1, 1, 3, 0);
    b7 = conv(b7, 192, 3, 3, 2, 2);
    return cat({b3, b7, maxp(x)});
  }
  ValueRef e(ValueRef x) {
    ValueRef b1 = conv(x, 320, 1, 1);
    ValueRef b3 = conv(x, 384, 1, 1);
    b3 = cat({conv(b3, 384, 1, 3, 1, 1, 0, 1), conv(b3, 384, 3, 1, 1, 1, 1, 0)});
    ValueRef bd = conv(conv(x, 448, 1, 1), 384, 3, 3, 1, 1, 1, 1);
    bd = cat({conv(bd, 384, 1, 3, 1, 1, 0, 1), conv(bd, 384, 3, 1, 1, 1, 1, 0)});
    ValueRef bp = conv(avg(x), 192, 1, 1);
    return cat({b1, b3, bd, bp});
  }
};
}  // namespace


ComputationGraph get_inception_v3_computation_graph(const InceptionV3ModelConfig& cfg) {
  ComputationGraph cg;
  Inception I{cg};
  ValueRef x = cg.create_input(TensorShape{{cfg.batch_size, 3, 299, 299}, DataType::FLOAT}, true, "input");
  x = I.conv(x, 32, 3, 3, 2, 2);
  x = I.conv(x, 32, 3, 3);
  x = I.conv(x, 64, 3, 3, 1, 1, 1, 1);
  x = I.maxp(x);
  x = I.conv(x, 80, 1, 1);
  x = I.conv(x, 192, 3, 3);
  x = I.maxp(x);
  x = I.a(x, 32);
  x = I.a(x, 64);
  x = I.a(x, 64);
  x = I.b(x);
  x = I.c(x, 128);
  x = I.c(x, 160);
  x = I.c(x, 160);
  x = I.c(x, 192);
  x = I.d(x);
  x = I.e(x);
  x = I.e(x);
  x = cg.pool2d(x, 8, 8, 1, 1, 0, 0, "avg", Activation::NONE, "avgpool");
  x = cg.flat(x, "flat");
  x = cg.dropout(x, 0.5, 0, "dropout");
  x = cg.dense(x, cfg.num_classes, Activation::NONE, true, "fc");
  cg.softmax(x, -1, "softmax");
  return cg;
}

// ---------------------------------------------------------------------------
CandleUnoModelConfig::CandleUnoModelConfig() {
  feature_shapes = {{"dose", 1}, {"cell.rnaseq", 942}, {"drug.descriptors", 5270}, {"drug.fingerprints", 2048}};
  input_features = {{"dose1", "dose"},
                    {"dose2", "dose"},
                    {"cell.rnaseq", "cell.rnaseq"},
                    {"drug1.descriptors", "drug.descriptors"},
                    {"drug1.fingerprints", "drug.fingerprints"},
                    {"drug2.descriptors", "drug.descriptors"},
                    {"drug2.fingerprints", "drug.fingerprints"}};
}

CandleUnoModelConfig CandleUnoModelConfig::from_json(const Json& j) {
  CandleUnoModelConfig c;
  get(j, "batch_size", c.batch_size);
  get(j, "dropout", c.dropout);
  get(j, "residual", c.residual);
  if (j.is_object() && j.contains("dense_layers")) c.dense_layers = j.at("dense_layers").as_int_vector();
  if (j.is_object() && j.contains("dense_feature_layers"))
    c.dense_feature_layers = j.at("dense_feature_layers").as_int_vector();
  if (j.is_object() && j.contains("feature_shapes")) {
    c.feature_shapes.clear();
    for (auto const& kv : j.at("feature_shapes").as_object()) c.feature_shapes[kv.first] = kv.second.as_int();
  }
  if (j.is_object() && j.contains("input_features")) {
    c.input_features.clear();
    for (auto const& kv : j.at("input_features").as_object()) c.input_features[kv.first] = kv.second.as_string();
  }
  return c;
}

Json CandleUnoModelConfig::to_json() const {
  Json j = Json::object();
  j["batch_size"] = batch_size;
  j["dense_layers"] = Json(dense_layers);
  j["dense_feature_layers"] = Json(dense_feature_layers);
  Json fs = Json::object();
  for (auto const& kv : feature_shapes) fs[kv.first] = kv.second;
  j["feature_shapes"] = fs;
  Json inf = Json::object();
  for (auto const& kv : input_features) inf[kv.first] = kv.second;
  j["input_features"] = inf;
  j["dropout"] = dropout;
  j["residual"] = residual;
  return j;
}

ComputationGraph get_candle_uno_computation_graph(const CandleUnoModelConfig& c) {
  ComputationGraph cg;
  std::set<std::string> tower_types;
  for (auto const& kv : c.feature_shapes) {
    auto dot = kv.first.find('.');
    if (dot == std::string::npos) continue;
    auto base = kv.first.substr(0, dot);
    if (base == "cell" || base == "drug") tower_types.insert(kv.first);
  }
  std::vector<ValueRef> encoded;
  for (auto const& kv : c.input_features) {
    int64_t width = c.feature_shapes.at(kv.second);
    ValueRef in = cg.create_input(TensorShape{{c.batch_size, width}, DataType::FLOAT}, true, kv.first);
    if (tower_types.count(kv.second)) {
      ValueRef t = in;
      int i = 0;
      for (int64_t d : c.dense_feature_layers) {
        std::string p = kv.first + ".tower" + std::to_string(i++);
        t = cg.dense(t, d, Activation::RELU, false, p, kGlorotNormal);
        if (c.dropout > 0) t = cg.dropout(t, c.dropout, 0, p + "_dropout");
      }
      encoded.push_back(t);
    } else {
      encoded.push_back(in);
    }
  }
  ValueRef out = cg.concat(encoded, 1, "concat");
  int i = 0;
  for (int64_t d : c.dense_layers) {
    std::string p = "dense" + std::to_string(i++);
    ValueRef res = out;
    out = cg.dense(out, d, Activation::RELU, false, p, kGlorotNormal);
    if (c.dropout > 0) out = cg.dropout(out, c.dropout, 0, p + "_dropout");
    if (c.residual && cg.shape(res) == cg.shape(out)) out = cg.binary(OpType::EW_ADD, out, res, p + "_residual");
  }
  cg.dense(out, 1, Activation::NONE, false, "out", kGlorotNormal);
  return cg;
}

// ---------------------------------------------------------------------------
ComputationGraph get_split_test_computation_graph(int64_t batch_size) {
  ComputationGraph cg;
  ValueRef t = cg.create_input(TensorShape{{batch_size, 256}, DataType::FLOAT}, true, "input");
  t = cg.unary(OpType::RELU, cg.dense(t, 128, Activation::NONE, true, "fc0"), "relu0");
  ValueRef a = cg.dense(t, 64, Activation::NONE, true, "fc1a");
  ValueRef b = cg.dense(t, 64, Activation::NONE, true, "fc1b");
  t = cg.unary(OpType::RELU, cg.binary(OpType::EW_ADD, a, b, "add1"), "relu1");
  a = cg.dense(t, 32, Activation::NONE, true, "fc2a");
  b = cg.dense(t, 32, Activation::NONE, true, "fc2b");
  t = cg.unary(OpType::RELU, cg.binary(OpType::EW_ADD, a, b, "add2"), "relu2");
  cg.softmax(t, -1, "softmax");
  return cg;
}

ComputationGraph get_single_operator_computation_graph(int64_t batch_size) {
  ComputationGraph cg;
  ValueRef t = cg.create_input(TensorShape{{batch_size, 1024}, DataType::FLOAT}, true, "input");
  cg.dense(t, 1024, Activation::NONE, true, "linear");
  return cg;
}

std::vector<std::string> model_names() {
  return {"transformer", "inception_v3", "candle_uno", "bert", "split_test", "single_operator"};
}

ComputationGraph get_model_computation_graph(const std::string& name, const Json& config) {
  if (name == "bert") return get_bert_computation_graph(BertModelConfig::from_json(config));
  if (name == "gpt") {
    auto c = BertModelConfig::from_json(config);
    c.causal = true;
    return get_bert_computation_graph(c);
  }
  if (name == "transformer") return get_transformer_computation_graph(TransformerModelConfig::from_json(config));
  if (name == "inception_v3") return get_inception_v3_computation_graph(InceptionV3ModelConfig::from_json(config));
  if (name == "candle_uno") return get_candle_uno_computation_graph(CandleUnoModelConfig::from_json(config));
  int64_t bs = 32;
  if (config.is_object() && config.contains("batch_size")) bs = config.at("batch_size").as_int();
  if (name == "split_test") return get_split_test_computation_graph(bs);
  if (name == "single_operator") return get_single_operator_computation_graph(bs);
  throw FFError("unknown model '" + name + "'");
}

}  // namespace ff
