// pgo_gtsam.hpp -- header-only C++ adapter: the GTSAM names that
// /root/reference/src/graph/src/graph.cpp uses, implemented over the C-ABI of
// pgo.h (libpgo.so).  A maintainer switches graph.cpp by replacing the GTSAM
// includes of graph.hpp:18-25 with this header and `gtsam::` with `pgo_gtsam::`
// (INTEGRATION.md shows the diff).  Errors surface as the GTSAM exception names.
#pragma once

#include <cmath>
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "pgo.h"

namespace pgo_gtsam {

using Key = std::uint64_t;  // gtsam::Key

struct ValuesKeyAlreadyExists : std::invalid_argument {
  using std::invalid_argument::invalid_argument;
};
struct ValuesKeyDoesNotExist : std::invalid_argument {
  using std::invalid_argument::invalid_argument;
};
struct IndeterminantLinearSystemException : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline void throw_status(int rc, const pgo_graph* g) {
  if (rc >= 0) return;
  const std::string msg = g ? pgo_last_error(g) : pgo_status_string(rc);
  switch (rc) {
    case PGO_E_DUP_KEY: throw ValuesKeyAlreadyExists(msg);
    case PGO_E_NO_KEY: throw ValuesKeyDoesNotExist(msg);
    case PGO_E_INDETERMINANT: throw IndeterminantLinearSystemException(msg);
    default: throw std::runtime_error(msg);
  }
}

// gtsam::Pose2 (graph.cpp:44,72,89-91)
class Pose2 {
 public:
  Pose2() = default;
  Pose2(double x, double y, double theta) : x_(x), y_(y), t_(theta) {}
  double x() const { return x_; }
  double y() const { return y_; }
  double theta() const { return std::atan2(std::sin(t_), std::cos(t_)); }
  double raw_theta() const { return t_; }

 private:
  double x_ = 0, y_ = 0, t_ = 0;
};

// Row-major 3x3, filled like covariance_to_eigen (graph.hpp:45-58) fills Q.
struct Matrix3 {
  double m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  double& operator()(int r, int c) { return m[3 * r + c]; }
  double operator()(int r, int c) const { return m[3 * r + c]; }
  static Matrix3 Zero() { return Matrix3(); }
};

namespace noiseModel {
struct Gaussian {
  Matrix3 cov;
  using shared_ptr = const Gaussian*;  // value semantics suffice here
  static Gaussian Covariance(const Matrix3& q) { return Gaussian{q}; }  // graph.cpp:45,83,103
};
}  // namespace noiseModel

template <class T>
struct PriorFactor {  // gtsam::PriorFactor<Pose2> (graph.cpp:57)
  Key key;
  T prior;
  noiseModel::Gaussian noise;
  PriorFactor(Key k, const T& p, const noiseModel::Gaussian& n) : key(k), prior(p), noise(n) {}
};

template <class T>
struct BetweenFactor {  // gtsam::BetweenFactor<Pose2> (graph.cpp:87-92,106-111)
  Key key1, key2;
  T measured;
  noiseModel::Gaussian noise;
  BetweenFactor(Key a, Key b, const T& z, const noiseModel::Gaussian& n) : key1(a), key2(b), measured(z), noise(n) {}
};

class Values {  // gtsam::Values restricted to Pose2
 public:
  void insert(Key k, const Pose2& p) {  // graph.cpp:58,86
    if (pos_.count(k)) throw ValuesKeyAlreadyExists("key " + std::to_string(k) + " already inserted");
    pos_[k] = keys_.size();
    keys_.push_back(k);
    poses_.push_back(p);
  }
  template <class T>
  const Pose2& at(Key k) const {  // graph.cpp:123-125
    auto it = pos_.find(k);
    if (it == pos_.end()) throw ValuesKeyDoesNotExist("key " + std::to_string(k) + " has no value");
    return poses_[it->second];
  }
  bool exists(Key k) const { return pos_.count(k) != 0; }
  size_t size() const { return keys_.size(); }
  const std::vector<Key>& keys() const { return keys_; }
  const std::vector<Pose2>& poses() const { return poses_; }

 private:
  std::map<Key, size_t> pos_;
  std::vector<Key> keys_;
  std::vector<Pose2> poses_;
};

class NonlinearFactorGraph {  // gtsam::NonlinearFactorGraph
 public:
  void add(const PriorFactor<Pose2>& f) { priors_.push_back(f); }
  void add(const BetweenFactor<Pose2>& f) { betweens_.push_back(f); }
  size_t nrFactors() const { return priors_.size() + betweens_.size(); }  // graph.cpp:60,94,112
  size_t size() const { return nrFactors(); }
  const std::vector<PriorFactor<Pose2>>& priors() const { return priors_; }
  const std::vector<BetweenFactor<Pose2>>& betweens() const { return betweens_; }

 private:
  std::vector<PriorFactor<Pose2>> priors_;
  std::vector<BetweenFactor<Pose2>> betweens_;
};

struct LevenbergMarquardtParams {
  pgo_params p;
  LevenbergMarquardtParams() { pgo_default_params(&p); }
};

// gtsam::LevenbergMarquardtOptimizer(graph, initial).optimize() (graph.cpp:119)
class LevenbergMarquardtOptimizer {
 public:
  LevenbergMarquardtOptimizer(const NonlinearFactorGraph& graph, const Values& initial,
                              const LevenbergMarquardtParams& params = LevenbergMarquardtParams(), int device = 0)
      : graph_(graph), initial_(initial), params_(params) {
    pgo_opts o{};
    o.device = device;
    g_ = pgo_create(&o);
    if (!g_) throw std::runtime_error("pgo_create failed");
  }
  ~LevenbergMarquardtOptimizer() { pgo_destroy(g_); }
  LevenbergMarquardtOptimizer(const LevenbergMarquardtOptimizer&) = delete;
  LevenbergMarquardtOptimizer& operator=(const LevenbergMarquardtOptimizer&) = delete;

  // GTSAM keeps the optimizer's state: a second optimize() continues from the
  // values the first one reached (defaultOptimize on state_), so the handle is
  // loaded once and later calls only re-run the solver on it.
  Values optimize() {
    if (!loaded_) load();
    throw_status(pgo_optimize(g_, &params_.p, &stats_), g_);
    Values out;
    std::vector<double> xyt(3 * initial_.size());
    throw_status(pgo_get_poses(g_, initial_.size(), nullptr, xyt.data()), g_);
    for (size_t i = 0; i < initial_.size(); i++)
      out.insert(initial_.keys()[i], Pose2(xyt[3 * i], xyt[3 * i + 1], xyt[3 * i + 2]));
    return out;
  }
  const pgo_stats& stats() const { return stats_; }
  int iterations() const { return stats_.iterations; }
  double error() const { return stats_.final_error; }

 private:
  void load() {
    for (size_t i = 0; i < initial_.size(); i++) {
      const Pose2& p = initial_.poses()[i];
      throw_status(pgo_add_vertex(g_, initial_.keys()[i], p.x(), p.y(), p.raw_theta()), g_);
    }
    for (const auto& f : graph_.priors()) {
      const double z[3] = {f.prior.x(), f.prior.y(), f.prior.raw_theta()};
      throw_status(pgo_add_prior(g_, f.key, z, f.noise.cov.m), g_);
    }
    for (const auto& f : graph_.betweens()) {
      const double z[3] = {f.measured.x(), f.measured.y(), f.measured.raw_theta()};
      throw_status(pgo_add_edge(g_, f.key1, f.key2, z, f.noise.cov.m), g_);
    }
    loaded_ = true;
  }

  const NonlinearFactorGraph& graph_;
  const Values& initial_;
  LevenbergMarquardtParams params_;
  pgo_graph* g_ = nullptr;
  pgo_stats stats_{};
  bool loaded_ = false;
};

// gtsam::Marginals(graph, values) (graph.cpp:120, commented in the reference):
// marginalCovariance(key) is the pose's 3x3 covariance (x, y, theta) at `values`,
// row-major in Matrix3::m (what eigen_to_covariance, graph.hpp:60-68, copies).
class Marginals {
 public:
  Marginals(const NonlinearFactorGraph& graph, const Values& values, int device = 0) {
    pgo_opts o{};
    o.device = device;
    g_ = pgo_create(&o);
    if (!g_) throw std::runtime_error("pgo_create failed");
    for (size_t i = 0; i < values.size(); i++) {
      const Pose2& p = values.poses()[i];
      throw_status(pgo_add_vertex(g_, values.keys()[i], p.x(), p.y(), p.raw_theta()), g_);
    }
    for (const auto& f : graph.priors()) {
      const double z[3] = {f.prior.x(), f.prior.y(), f.prior.raw_theta()};
      throw_status(pgo_add_prior(g_, f.key, z, f.noise.cov.m), g_);
    }
    for (const auto& f : graph.betweens()) {
      const double z[3] = {f.measured.x(), f.measured.y(), f.measured.raw_theta()};
      throw_status(pgo_add_edge(g_, f.key1, f.key2, z, f.noise.cov.m), g_);
    }
  }
  ~Marginals() { pgo_destroy(g_); }
  Marginals(const Marginals&) = delete;
  Marginals& operator=(const Marginals&) = delete;

  Matrix3 marginalCovariance(Key key) const {
    Matrix3 out;
    throw_status(pgo_marginal_covariances(g_, 1, &key, out.m), g_);
    return out;
  }

 private:
  pgo_graph* g_ = nullptr;
};

}  // namespace pgo_gtsam
