// ffc-substitution-to-dot: render one rule of a legacy substitution corpus
// (graph_subst JSON) as graphviz, or list the rules.
//
// Parity: bin/substitution-to-dot/substitution_to_dot.cc:17-152
//   substitution-to-dot <rules.json> <rule name | index>
//   substitution-to-dot <rules.json> --list
#include <fstream>
#include <iostream>
#include <sstream>

#include "ff/substitution.h"

using namespace ff;

int main(int argc, char** argv) {
  if (argc < 3) {
    std::cerr << "usage: ffc-substitution-to-dot RULES.json (RULE_NAME | INDEX | --list | --convertible)\n";
    return 2;
  }
  std::ifstream f(argv[1]);
  if (!f) {
    std::cerr << "error: cannot open " << argv[1] << "\n";
    return 1;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  try {
    auto coll = load_legacy_rules(Json::parse(ss.str()));
    std::string sel = argv[2];
    if (sel == "--list") {
      for (size_t i = 0; i < coll.rules.size(); ++i) {
        auto const& r = coll.rules[i];
        std::cout << i << "\t" << r.name << "\t" << r.src.size() << "->" << r.dst.size() << "\n";
      }
      return 0;
    }
    if (sel == "--convertible") {
      size_t n = 0;
      for (auto const& r : coll.rules) n += substitution_from_legacy_rule(r).has_value() ? 1 : 0;
      std::cout << n << " / " << coll.rules.size() << " rules convertible to PCG substitutions\n";
      return 0;
    }
    for (size_t i = 0; i < coll.rules.size(); ++i) {
      if (coll.rules[i].name == sel || std::to_string(i) == sel) {
        std::cout << legacy_rule_to_dot(coll.rules[i]);
        return 0;
      }
    }
    std::cerr << "error: no rule '" << sel << "'\n";
    return 1;
  } catch (const std::exception& e) {
    std::cerr << "error: " << e.what() << "\n";
    return 1;
  }
}
