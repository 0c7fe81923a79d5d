#include "ff/search.h"
#include "ff/memory_plan.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <limits>
#include <atomic>
#include <functional>
#include <mutex>
#include <optional>
#include <thread>
#include <queue>
#include <random>
#include <unordered_set>

namespace ff {

static constexpr double kInf = std::numeric_limits<double>::infinity();

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

Json SearchResult::to_json(const ComputationGraph* cg) const {
  Json j = Json::object();
  j["algorithm"] = algorithm;
  j["cost"] = cost;
  j["data_parallel_cost"] = data_parallel_cost;
  if (unmapped_cost >= 0) j["unmapped_cost"] = unmapped_cost;
  j["predicted_speedup_over_dp"] = cost > 0 ? data_parallel_cost / cost : 0.0;
  j["iterations"] = iterations;
  j["evaluated"] = evaluated;
  j["accepted"] = accepted;
  j["elapsed"] = elapsed;
  j["time_limited"] = time_limited;
  j["trace"] = trace;
  if (rules) {
    j["rules"] = static_cast<int64_t>(rules);
    j["rule_set_rules"] = static_cast<int64_t>(rule_set_rules);
    Json br = Json::array();
    for (auto const& n : best_rules) br.push_back(n);
    j["best_rules"] = br;
    j["mapping_cache_entries"] = mapping_cache_entries;
    j["mapping_cache_hits"] = mapping_cache_hits;
    j["mapped_states"] = mapped_states;
  }
  j["micro_batches"] = static_cast<int64_t>(micro_batches);
  if (pipeline_stages > 0) j["pipeline_stages"] = static_cast<int64_t>(pipeline_stages);
  if (!pipeline.as_array().empty()) j["pipeline_candidates"] = pipeline;
  if (memory_plan.is_object()) j["memory_plan"] = memory_plan;
  if (cg && !strategy.empty()) j["strategy"] = strategy_to_json(*cg, strategy);
  Json v = Json::object();
  for (auto const& kv : views) v[std::to_string(kv.first)] = Json(std::vector<int64_t>(kv.second.begin(), kv.second.end()));
  j["views"] = v;
  return j;
}

double evaluate_strategy(const ComputationGraph& cg, const StrategyConfig& s, const CostModel& cm,
                         const SimConfig& sim, int world, SimResult* out) {
  try {
    auto L = lower_strategy(cg, s, world);
    SimConfig c = sim;
    c.world = world;
    Simulator S(cm, c);
    auto r = S.simulate(L.pcg);
    if (out) *out = r;
    return r.iteration_time;
  } catch (const FFError&) {
    return kInf;
  }
}

static std::string layer_signature(const ComputationGraph& cg, int id) {
  std::string s = cg.g.node(id).label.op.str();
  for (auto const& v : cg.layer_data_inputs(id)) s += "|" + cg.shape(v).str();
  return s;
}

SearchResult mcmc_search(const ComputationGraph& cg, const CostModel& cm, const SearchConfig& cfg,
                         const StrategyConfig* initial) {
  const double t0 = now_s();
  SearchResult R;
  R.algorithm = "mcmc";
  R.trace = Json::array();
  const int world = cfg.world;
  std::mt19937_64 rng(cfg.seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);

  std::vector<int> layers;
  std::map<int, std::vector<LayerConfig>> cands;
  std::map<std::string, std::vector<int>> groups;
  std::map<int, std::string> sig;
  for (int id : cg.g.topo_order()) {
    auto t = cg.g.node(id).label.op.type;
    if (t == OpType::WEIGHT) continue;
    cands[id] = candidate_configs(cg, id, world, cfg.space);
    if (cands[id].size() > 1) layers.push_back(id);
    sig[id] = layer_signature(cg, id);
    groups[sig[id]].push_back(id);
  }
  StrategyConfig dp = data_parallel_strategy(cg, world);
  SimConfig sim = cfg.sim;
  sim.world = world;
  R.data_parallel_cost = evaluate_strategy(cg, dp, cm, sim, world);
  StrategyConfig cur = initial ? *initial : dp;
  double cur_cost = initial ? evaluate_strategy(cg, cur, cm, sim, world) : R.data_parallel_cost;
  StrategyConfig best = cur;
  double best_cost = cur_cost;
  R.evaluated = 2;
  R.trace.push_back(Json(std::vector<double>{0.0, best_cost}));
  int it = 0;
  for (; it < cfg.budget && !layers.empty(); ++it) {
    if (now_s() - t0 > cfg.time_limit) {
      R.time_limited = true;
      break;
    }
    int id = layers[rng() % layers.size()];
    auto const& cs = cands[id];
    LayerConfig c = cs[rng() % cs.size()];
    if (c == cur[id]) continue;
    StrategyConfig next = cur;
    if (U(rng) < cfg.group_move_prob) {
      for (int g : groups[sig[id]]) next[g] = c;
    } else {
      next[id] = c;
    }
    double nc = evaluate_strategy(cg, next, cm, sim, world);
    ++R.evaluated;
    if (!std::isfinite(nc)) continue;
    bool accept = nc < cur_cost || U(rng) < std::exp(-cfg.mcmc_beta * (nc - cur_cost) / cur_cost);
    if (accept) {
      cur = std::move(next);
      cur_cost = nc;
      ++R.accepted;
      if (cur_cost < best_cost) {
        best = cur;
        best_cost = cur_cost;
        R.trace.push_back(Json(std::vector<double>{static_cast<double>(it), best_cost}));
      }
    }
  }
  R.iterations = it;
  R.strategy = best;
  R.cost = best_cost;
  R.pcg = lower_strategy(cg, best, world).pcg;
  R.elapsed = now_s() - t0;
  return R;
}

// Every tensor's degrees must fit the devices the executor has.
static bool fits_world(const ParallelComputationGraph& g, int world) {
  for (auto const& v : g.g.all_values()) {
    int t = g.shape(v).total_parallel_degree();
    if (t > world || world % t != 0) return false;
  }
  return true;
}

namespace {
struct State {
  double cost;
  int id;
  bool operator>(const State& o) const { return cost > o.cost; }
};
}  // namespace

SearchResult unity_search(const ParallelComputationGraph& initial, const CostModel& cm, const SearchConfig& cfg,
                          const std::vector<Substitution>& extra_rules) {
  const double t0 = now_s();
  SearchResult R;
  R.algorithm = "unity";
  R.trace = Json::array();
  SimConfig sim = cfg.sim;
  sim.world = cfg.world;
  Simulator S(cm, sim);
  // joint search (unity_algorithm.cc:37-90): every state is priced with its
  // own DP machine mapping, through ONE mapping cache keyed by subtree
  // content, so a rewrite re-solves only the subtrees it changed
  MMCache mm_cache;
  double best_so_far = kInf;
  int mapped_states = 0;
  // whole-world price (thread-safe: the cost model memoises under a mutex)
  auto whole_cost = [&](const ParallelComputationGraph& g) -> double {
    try {
      return S.simulate(g).iteration_time;
    } catch (const FFError&) {
      return kInf;
    }
  };
  // the DP mapping (~0.1-0.5 s on a BERT-large PCG) for every state whose
  // whole-world cost is within mapping_alpha of the best so far: the states
  // the queue can still pop ahead of the best.  Runs in candidate order on
  // one thread (the cache is shared), so the search stays deterministic.
  auto mapped_cost = [&](const ParallelComputationGraph& g, double whole, std::map<int, Placement>* views) -> double {
    if (views) views->clear();
    if (!std::isfinite(whole)) return whole;
    try {
      if (cfg.use_machine_mapping && cfg.world > 1 && whole <= best_so_far * cfg.mapping_alpha &&
          (cfg.max_mapped_states < 0 || mapped_states < cfg.max_mapped_states)) {
        auto m = get_optimal_machine_mapping(g, cm, cfg.world, MachineMappingOptions{}, &mm_cache);
        ++mapped_states;
        if (m.feasible) {
          // the simulator prices the mapped placements against the
          // whole-world ones (the DP's per-op sum has no overlap); the better
          // one is the state's cost and placement
          const double mapped = S.simulate(g, m.views).iteration_time;
          if (mapped < whole) {
            if (views) *views = m.views;
            best_so_far = std::min(best_so_far, mapped);
            return mapped;
          }
        }
      }
    } catch (const FFError&) {
    }
    best_so_far = std::min(best_so_far, whole);
    return whole;
  };
  auto rules = generate_parallelization_substitutions(initial, cfg.world);
  rules.insert(rules.end(), extra_rules.begin(), extra_rules.end());
  if (!cfg.substitution_path.empty()) {
    auto const& rs = cached_substitutions(cfg.substitution_path);
    rules.insert(rules.end(), rs.begin(), rs.end());
    R.rule_set_rules = static_cast<int>(rs.size());
  }
  R.rules = static_cast<int>(rules.size());
  // candidate rewrites of a popped state are applied, checked, hashed and
  // priced on a pool of threads (FF_SEARCH_THREADS, default up to 16): one
  // pop of a 24-layer BERT-large PCG expands ~10^3 rewrites, each a graph
  // copy + hash + simulation.  A network model with its own route cache
  // (not thread-safe) keeps the search on one thread.
  int nthreads = static_cast<int>(std::thread::hardware_concurrency());
  if (const char* e = getenv("FF_SEARCH_THREADS")) nthreads = std::atoi(e);
  nthreads = std::max(1, std::min(nthreads, 16));
  if (sim.network) nthreads = 1;
  auto parallel_for = [&](size_t n, const std::function<void(size_t)>& fn) {
    if (nthreads <= 1 || n < 2) {
      for (size_t i = 0; i < n; ++i) fn(i);
      return;
    }
    std::atomic<size_t> next{0};
    std::vector<std::thread> pool;
    const int T = static_cast<int>(std::min<size_t>(nthreads, n));
    for (int t = 0; t < T; ++t)
      pool.emplace_back([&] {
        for (size_t i = next.fetch_add(1); i < n; i = next.fetch_add(1)) fn(i);
      });
    for (auto& th : pool) th.join();
  };

  std::vector<ParallelComputationGraph> states;
  std::vector<std::pair<int, int>> parent;   // state -> (parent state, rule index)
  parent.push_back({-1, -1});
  std::vector<std::map<int, Placement>> state_views;
  std::priority_queue<State, std::vector<State>, std::greater<State>> pq;
  std::unordered_set<size_t> seen;
  states.push_back(initial);
  state_views.emplace_back();
  double c0 = mapped_cost(initial, whole_cost(initial), &state_views[0]);
  R.data_parallel_cost = c0;
  pq.push({c0, 0});
  seen.insert(initial.structural_hash());
  int best = 0;
  double best_cost = c0;
  R.evaluated = 1;
  R.trace.push_back(Json(std::vector<double>{0.0, best_cost}));
  int it = 0;
  double prof[5] = {0, 0, 0, 0, 0};
  bool timed_out = false;
  struct Cand {
    int rule;
    const PCGPatternMatch* match;
    std::optional<ParallelComputationGraph> g;
    size_t hash = 0;
    bool ok = false;
    double whole = kInf;
  };
  for (; it < cfg.budget && !pq.empty(); ++it) {
    if (now_s() - t0 > cfg.time_limit) {
      timed_out = true;
      break;
    }
    State s = pq.top();
    pq.pop();
    if (s.cost < best_cost) {
      best_cost = s.cost;
      best = s.id;
      R.trace.push_back(Json(std::vector<double>{static_cast<double>(it), best_cost}));
    } else if (s.cost > best_cost * cfg.alpha) {
      continue;
    }
    const ParallelComputationGraph cur = states[s.id];
    const PatternMatchIndex ix(cur);
    // every (rule, match) of this state, in rule order
    double tm = now_s();
    std::vector<std::vector<PCGPatternMatch>> matches(rules.size());
    for (size_t ri = 0; ri < rules.size(); ++ri) matches[ri] = find_pattern_matches(rules[ri].pattern, cur, ix, 4096);
    std::vector<Cand> cands;
    for (size_t ri = 0; ri < rules.size(); ++ri)
      for (auto const& m : matches[ri]) cands.push_back(Cand{static_cast<int>(ri), &m, std::nullopt});
    prof[4] += now_s() - tm;
    // apply + checks + hash, in parallel
    double ta = now_s();
    parallel_for(cands.size(), [&](size_t i) {
      if (now_s() - t0 > cfg.time_limit) return;
      Cand& c = cands[i];
      auto next = apply_substitution(cur, rules[c.rule], *c.match);
      if (!next || next->num_operator_nodes() > cfg.max_num_ops || !fits_world(*next, cfg.world)) return;
      c.hash = next->structural_hash();
      c.g = std::move(next);
      c.ok = true;
    });
    prof[0] += now_s() - ta;
    // dedupe in candidate order (deterministic), then price the new ones in parallel
    std::vector<size_t> fresh;
    for (size_t i = 0; i < cands.size(); ++i)
      if (cands[i].ok && seen.insert(cands[i].hash).second) fresh.push_back(i);
    ta = now_s();
    parallel_for(fresh.size(), [&](size_t k) {
      if (now_s() - t0 > cfg.time_limit) return;
      Cand& c = cands[fresh[k]];
      c.whole = whole_cost(*c.g);
    });
    prof[3] += now_s() - ta;
    ta = now_s();
    for (size_t i : fresh) {
      Cand& c = cands[i];
      if (!std::isfinite(c.whole)) continue;   // failed, or not priced before the time limit
      std::map<int, Placement> v;
      const double cst = mapped_cost(*c.g, c.whole, &v);
      ++R.evaluated;
      if (!std::isfinite(cst) || cst > cfg.threshold) continue;
      states.push_back(std::move(*c.g));
      parent.push_back({s.id, c.rule});
      state_views.push_back(std::move(v));
      pq.push({cst, static_cast<int>(states.size()) - 1});
      if (cst < best_cost) {
        best_cost = cst;
        best = static_cast<int>(states.size()) - 1;
        R.trace.push_back(Json(std::vector<double>{static_cast<double>(it), best_cost}));
      }
    }
    prof[2] += now_s() - ta;
    if (now_s() - t0 > cfg.time_limit) {
      timed_out = true;
      ++it;
      break;
    }
  }
  if (getenv("FF_SEARCH_PROFILE"))
    fprintf(stderr, "unity: %d threads, apply+hash %.2fs price %.2fs map+insert %.2fs match %.2fs total %.2fs, "
            "%d pops, %d evaluated, %zu states%s\n", nthreads, prof[0], prof[3], prof[2], prof[4], now_s() - t0, it,
            R.evaluated, states.size(), timed_out ? " (time limit)" : "");
  R.iterations = it;
  R.time_limited = timed_out;
  R.mapping_cache_entries = static_cast<int64_t>(mm_cache.results.size());
  R.mapping_cache_hits = static_cast<int64_t>(mm_cache.hits);
  R.mapped_states = mapped_states;
  R.pcg = states[best];
  R.views = state_views[best];
  R.cost = best_cost;
  for (int k = best; k >= 0 && parent[k].second >= 0; k = parent[k].first)
    R.best_rules.insert(R.best_rules.begin(), rules[parent[k].second].name);
  R.elapsed = now_s() - t0;
  return R;
}

const std::vector<Substitution>& cached_substitutions(const std::string& path) {
  static std::mutex mu;
  static std::map<std::string, std::vector<Substitution>> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(path);
  if (it == cache.end()) it = cache.emplace(path, load_substitutions_file(path)).first;
  return it->second;
}

SearchResult graph_optimize(const ComputationGraph& cg, const CostModel& cm, const SearchConfig& cfg) {
  const double t0 = now_s();
  SearchConfig mc = cfg;
  mc.time_limit = cfg.time_limit * cfg.mcmc_time_share;
  auto m = mcmc_search(cg, cm, mc);
  SearchConfig uc = cfg;
  uc.time_limit = std::max(0.0, cfg.time_limit - (now_s() - t0));
  uc.budget = cfg.unity_budget >= 0 ? cfg.unity_budget : cfg.budget;
  SearchResult best = m;
  if (uc.time_limit > 0.05 && uc.budget > 0) {
    auto u = unity_search(m.pcg, cm, uc);
    best.rules = u.rules;
    best.rule_set_rules = u.rule_set_rules;
    best.mapping_cache_entries = u.mapping_cache_entries;
    best.mapping_cache_hits = u.mapping_cache_hits;
    best.mapped_states = u.mapped_states;
    const int evaluated = m.evaluated + u.evaluated;
    const bool limited = m.time_limited || u.time_limited;
    if (u.cost < best.cost * 0.999) {
      u.data_parallel_cost = m.data_parallel_cost;
      u.strategy.clear();
      u.algorithm = "mcmc+unity";
      best = u;
    }
    best.evaluated = evaluated;   // every strategy / state priced by either phase
    best.time_limited = limited;
  } else if (uc.budget > 0) {
    best.time_limited = true;     // the MCMC phase left Unity no time
  }
  // final machine mapping (the reference's Unity cost is the mapping DP's;
  // here per-state costs use whole-world placements and the DP, ~0.1 s on a
  // BERT-large PCG, runs once on the winner)
  if (cfg.final_machine_mapping && cfg.world > 1 && best.views.empty()) {
    try {
      auto mm = get_optimal_machine_mapping(best.pcg, cm, cfg.world);
      if (mm.feasible) {
        SimConfig sim = cfg.sim;
        sim.world = cfg.world;
        const double c = Simulator(cm, sim).simulate(best.pcg, mm.views).iteration_time;
        best.unmapped_cost = best.cost;
        if (c < best.cost * 0.99) {
          best.views = mm.views;
          best.cost = c;
          best.algorithm += "+mapping";
        }
      }
    } catch (const FFError&) {
    }
  }
  // pipeline parallelism: stage cuts x micro-batches, at equal work
  if (cfg.pipeline && cfg.world > 1) {
    const int M = std::max(1, cfg.micro_batches);
    SimConfig sim = cfg.sim;
    sim.world = cfg.world;
    Simulator S(cm, sim);
    try {
      double t_best = micro_batched_step_time(S.simulate(best.pcg, best.views), M);
      const double t_dp = micro_batched_step_time(S.simulate(data_parallel_pcg(cg, cfg.world)), M);
      if (M > 1 && t_dp < t_best * 0.999) {
        // the winner of the one-batch search loses to DP once its forward /
        // backward repeats M times per synchronisation: keep DP
        best.pcg = data_parallel_pcg(cg, cfg.world);
        best.views.clear();
        best.strategy.clear();
        best.algorithm += "+dp_at_micro_batches";
        t_best = t_dp;
      }
      const PipelinePlan* win = nullptr;
      auto cands = pipeline_candidates(cg, cm, cfg.world, M, sim);
      Json list = Json::array();
      for (auto const& p : cands) {
        list.push_back(p.to_json());
        if (p.step_time < t_best * 0.99 && (!win || p.step_time < win->step_time)) win = &p;
      }
      best.pipeline = list;
      best.micro_batches = M;
      double chosen = t_best;
      if (win) {
        best.pcg = win->pcg;
        best.views = win->views;
        best.pipeline_stages = win->stages;
        best.strategy.clear();
        best.algorithm += "+pipeline";
        chosen = win->step_time;
      }
      if (M > 1 || win) {   // per micro-batch of an M-micro-batch step
        best.cost = chosen / M;
        best.data_parallel_cost = t_dp / M;
      }
    } catch (const FFError&) {
    }
  }
  // liveness memory plan of the winner: the busiest device's arena.  A
  // winner that does not fit the HBM is replaced by the fastest candidate
  // that does -- data parallelism or a pipeline split (stages hold 1/S of the
  // weights) -- so the 288 GB budget is checked by the search
  try {
    auto busiest = [](const std::vector<MemoryPlan>& ps) {
      double a = 0;
      for (auto const& p : ps) a = std::max(a, p.arena_bytes);
      return a;
    };
    // the executor's storage: bf16 activations / gradients when the cost
    // model prices bf16 compute, its fusions and saved tensors
    MemoryPlanConfig base_mc;
    base_mc.executor_fusions = cfg.sim.executor_fusions;
    base_mc.act_elem_bytes = cfg.sim.bf16_weight_grads ? 2.0 : 0.0;
    auto with_base = [&](MemoryPlanConfig c) {
      c.executor_fusions = base_mc.executor_fusions;
      c.act_elem_bytes = base_mc.act_elem_bytes;
      return c;
    };
    // a pipeline winner keeps several micro-batches of activations per stage
    MemoryPlanConfig best_mc = base_mc;
    if (best.pipeline_stages > 1) {
      SimConfig psim = cfg.sim;
      psim.world = cfg.world;
      for (auto& pl : pipeline_candidates(cg, cm, cfg.world, std::max(1, cfg.micro_batches), psim))
        if (pl.stages == best.pipeline_stages) best_mc = with_base(pipeline_memory_config(pl));
    }
    auto plans = plan_memory(best.pcg, best.views, cfg.world, best_mc);
    const double cap = cm.spec().hbm_capacity;
    if (cap > 0 && busiest(plans) > cap && cfg.world > 1) {
      SimConfig sim = cfg.sim;
      sim.world = cfg.world;
      const int M = std::max(1, cfg.micro_batches);
      Simulator S(cm, sim);
      double best_t = std::numeric_limits<double>::infinity();
      auto dp = data_parallel_pcg(cg, cfg.world);
      auto dplans = plan_memory(dp, {}, cfg.world, base_mc);
      bool found = false;
      ParallelComputationGraph fb_pcg;
      std::map<int, Placement> fb_views;
      std::vector<MemoryPlan> fb_plans;
      std::string tag;
      int stages = 0;
      if (busiest(dplans) <= cap) {
        best_t = micro_batched_step_time(S.simulate(dp), M);
        fb_pcg = dp;
        fb_plans = dplans;
        tag = "+memory_fallback_dp";
        found = true;
      }
      for (auto& pl : pipeline_candidates(cg, cm, cfg.world, M, sim)) {
        auto pp = plan_memory(pl.pcg, pl.views, cfg.world, with_base(pipeline_memory_config(pl)));
        if (busiest(pp) <= cap && pl.step_time < best_t) {
          best_t = pl.step_time;
          fb_pcg = pl.pcg;
          fb_views = pl.views;
          fb_plans = pp;
          tag = "+memory_fallback_pipeline";
          stages = pl.stages;
          found = true;
        }
      }
      if (found) {
        best.pcg = fb_pcg;
        best.views = fb_views;
        best.strategy.clear();
        best.cost = best_t / M;
        best.pipeline_stages = stages;
        best.algorithm += tag;
        plans = fb_plans;
      }
    }
    Json mp = Json::object();
    double arena = 0, live = 0, weights = 0, naive = 0;
    for (auto const& p : plans) {
      arena = std::max(arena, p.arena_bytes);
      live = std::max(live, p.peak_live_bytes);
      weights = std::max(weights, p.weight_bytes);
      naive = std::max(naive, p.naive_bytes);
    }
    mp["arena_bytes"] = arena;
    mp["peak_live_bytes"] = live;
    mp["weight_bytes"] = weights;
    mp["naive_bytes"] = naive;
    mp["devices"] = static_cast<int64_t>(plans.size());
    mp["fits_hbm"] = arena <= cm.spec().hbm_capacity;
    best.memory_plan = mp;
  } catch (const FFError&) {
  }
  best.elapsed = now_s() - t0;
  return best;
}

// JSON configuration (Python bindings, C FFI, CLIs)
SimConfig sim_config_from_json(const Json& j) {
  SimConfig c;
  if (!j.is_object()) return c;
  auto gi = [&](const char* k, int& v) { if (j.contains(k)) v = static_cast<int>(j.at(k).as_int()); };
  auto gd = [&](const char* k, double& v) { if (j.contains(k)) v = j.at(k).as_double(); };
  auto gb = [&](const char* k, bool& v) { if (j.contains(k)) v = j.at(k).as_bool(); };
  gi("world", c.world);
  gb("overlap_grad_sync", c.overlap_grad_sync);
  gd("bucket_bytes", c.bucket_bytes);
  gb("include_update", c.include_update);
  gd("update_bytes_per_param", c.update_bytes_per_param);
  gd("memory_penalty_per_mb", c.memory_penalty_per_mb);
  gd("comm_compute_slowdown", c.comm_compute_slowdown);
  gb("bf16_weight_grads", c.bf16_weight_grads);
  gb("parameter_server", c.parameter_server);
  gb("sparse_embedding_update", c.sparse_embedding_update);
  gb("executor_fusions", c.executor_fusions);
  return c;
}

SearchConfig search_config_from_json(const Json& j) {
  SearchConfig c;
  auto gi = [&](const char* k, int& v) { if (j.contains(k)) v = static_cast<int>(j.at(k).as_int()); };
  auto gd = [&](const char* k, double& v) { if (j.contains(k)) v = j.at(k).as_double(); };
  auto gb = [&](const char* k, bool& v) { if (j.contains(k)) v = j.at(k).as_bool(); };
  gi("world", c.world);
  gi("budget", c.budget);
  gd("alpha", c.alpha);
  gd("threshold", c.threshold);
  gi("max_num_ops", c.max_num_ops);
  gd("mcmc_beta", c.mcmc_beta);
  gd("group_move_prob", c.group_move_prob);
  if (j.contains("seed")) c.seed = static_cast<uint64_t>(j.at("seed").as_int());
  gd("time_limit", c.time_limit);
  gb("use_machine_mapping", c.use_machine_mapping);
  gd("mapping_alpha", c.mapping_alpha);
  gb("pipeline", c.pipeline);
  gi("micro_batches", c.micro_batches);
  gi("max_mapped_states", c.max_mapped_states);
  gb("final_machine_mapping", c.final_machine_mapping);
  gi("unity_budget", c.unity_budget);
  gd("mcmc_time_share", c.mcmc_time_share);
  if (j.contains("substitution_path")) c.substitution_path = j.at("substitution_path").as_string();
  gb("enable_parameter_parallel", c.space.enable_parameter_parallel);
  gb("enable_attribute_parallel", c.space.enable_attribute_parallel);
  gb("allow_partial_world", c.space.allow_partial_world);
  gi("max_model_degree", c.space.max_model_degree);
  if (j.contains("sim")) c.sim = sim_config_from_json(j.at("sim"));
  c.sim.world = c.world;
  return c;
}

}  // namespace ff
