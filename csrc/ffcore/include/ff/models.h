// Model builders producing ComputationGraphs (used by export-model-arch,
// the search benchmarks and the C++ tests).
//
// Parity: lib/models/src/models/{bert,transformer,inception_v3,candle_uno,
// split_test}/*.cc — same layer structure and defaults:
//  * BERT: bert.cc:25-158 (encoder on hidden states + vocab projection)
//  * Transformer: transformer.cc (6+6 layers, 512 features, FF 2048, 8 heads)
//  * InceptionV3: inception_v3.cc (299x299, stem + A x3, B, C x4, D, E x2)
//  * CANDLE-Uno: candle_uno.cc (feature towers 8x4192, dense 4x4192)
//  * split_test: split_test.cc:6-37
// Deliberate difference: attention head dims are hidden/heads (the usual
// BERT/Transformer definition); the reference passes dim_feedforward/heads.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "ff/computation_graph.h"
#include "ff/json.h"

namespace ff {

struct BertModelConfig {
  int64_t vocab_size = 30522, hidden_size = 768, num_encoder_layers = 12, num_heads = 12,
          dim_feedforward = 3072, sequence_length = 512, batch_size = 64;
  std::string hidden_act = "gelu";
  double hidden_dropout_prob = 0.1, attention_probs_dropout_prob = 0.1, initializer_range = 0.02,
         layer_norm_eps = 1e-12;
  bool causal = false;  // GPT-style decoder-only variant
  static BertModelConfig from_json(const Json& j);
  Json to_json() const;
};

struct TransformerModelConfig {
  int64_t num_features = 512, sequence_length = 512, batch_size = 64, dim_feedforward = 2048, num_heads = 8,
          num_encoder_layers = 6, num_decoder_layers = 6, vocab_size = 64;
  double dropout = 0.1, layer_norm_eps = 1e-5;
  static TransformerModelConfig from_json(const Json& j);
  Json to_json() const;
};

struct InceptionV3ModelConfig {
  int64_t num_classes = 1000, batch_size = 64;
  bool aux_logits = false;
  static InceptionV3ModelConfig from_json(const Json& j);
  Json to_json() const;
};

struct CandleUnoModelConfig {
  int64_t batch_size = 64;
  std::vector<int64_t> dense_layers = std::vector<int64_t>(4, 4192);
  std::vector<int64_t> dense_feature_layers = std::vector<int64_t>(8, 4192);
  std::map<std::string, int64_t> feature_shapes;
  std::map<std::string, std::string> input_features;
  double dropout = 0.1;
  bool residual = false;
  CandleUnoModelConfig();
  static CandleUnoModelConfig from_json(const Json& j);
  Json to_json() const;
};

ComputationGraph get_bert_computation_graph(const BertModelConfig& c);
ComputationGraph get_transformer_computation_graph(const TransformerModelConfig& c);
ComputationGraph get_inception_v3_computation_graph(const InceptionV3ModelConfig& c);
ComputationGraph get_candle_uno_computation_graph(const CandleUnoModelConfig& c);
ComputationGraph get_split_test_computation_graph(int64_t batch_size);
// A one-operator graph (export-model-arch "single_operator").
ComputationGraph get_single_operator_computation_graph(int64_t batch_size);

// Dispatch by name with an optional JSON config override.
ComputationGraph get_model_computation_graph(const std::string& name, const Json& config);
std::vector<std::string> model_names();

}  // namespace ff
