// ffc-export-model-arch: export a model's ComputationGraph (and optionally its
// series-parallel decomposition) as JSON, or render it as graphviz.
//
// Parity: bin/export-model-arch/src/export_model_arch.cc:21-220
//   export-model-arch {transformer, inception_v3, candle_uno, bert, split_test,
//                      single_operator} [--sp-decomposition] [--dot]
//                     [--preprocessed-dot]
// Output JSON: {"computation_graph": <cg v1>, "sp_decomposition": <tree|null>}
// Extra: --config '<json>' overrides the model config (e.g. '{"batch_size":8}').
#include <cstring>
#include <iostream>
#include <string>

#include "ff/models.h"
#include "ff/sp.h"

using namespace ff;

static int usage() {
  std::cerr << "usage: ffc-export-model-arch MODEL [--sp-decomposition] [--dot] [--preprocessed-dot] "
               "[--config JSON]\n  models:";
  for (auto const& m : model_names()) std::cerr << " " << m;
  std::cerr << " gpt\n";
  return 2;
}

int main(int argc, char** argv) {
  if (argc < 2) return usage();
  std::string model = argv[1];
  if (model == "-h" || model == "--help") return usage();
  bool sp = false, dot = false, pre_dot = false;
  Json config = Json::object();
  for (int i = 2; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--sp-decomposition") sp = true;
    else if (a == "--dot") dot = true;
    else if (a == "--preprocessed-dot") pre_dot = true;
    else if (a == "--config" && i + 1 < argc) config = Json::parse(argv[++i]);
    else return usage();
  }
  try {
    ComputationGraph cg = get_model_computation_graph(model, config);
    if (dot) {
      std::cout << cg.as_dot();
      return 0;
    }
    // SP preprocessing (reference: plain SP first, then drop weight sources)
    DiGraph g = cg.g.digraph();
    std::set<int> keep;
    for (int id : g.nodes)
      if (cg.g.node(id).label.op.type != OpType::WEIGHT) keep.insert(id);
    DiGraph pre = g.induced_subgraph(keep);
    if (pre_dot) {
      std::cout << digraph_as_dot(pre, [&](int n) { return cg.g.node(n).label.name; });
      return 0;
    }
    Json out = Json::object();
    out["computation_graph"] = cg.to_json();
    if (sp) {
      auto t = get_series_parallel_decomposition(g);
      if (!t) t = get_series_parallel_decomposition(pre);
      out["sp_decomposition"] = t ? t->to_json() : Json();
      if (!t) out["sp_decomposition_relaxed"] = get_relaxed_sp_decomposition(pre).to_json();
    } else {
      out["sp_decomposition"] = Json();
    }
    std::cout << out.dump(2) << "\n";
  } catch (const std::exception& e) {
    std::cerr << "error: " << e.what() << "\n";
    return 1;
  }
  return 0;
}
