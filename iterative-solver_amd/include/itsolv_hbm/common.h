// Solver bookkeeping shared by all layers: Logger levels (reference itsolv/Logger.h:40-69),
// Statistics (reference itsolv/Statistics.h:10-37), Verbosity and Options (reference itsolv/Options.h,
// LinearEigensystemDavidsonOptions.h, NonLinearEquationsDIISOptions.h) with the reference's option
// names parsed from "key=value,key=value" strings (reference itsolv/util.cpp:38-56).
#pragma once
#include <algorithm>
#include <cctype>
#include <iomanip>
#include <iostream>
#include <map>
#include <memory>
#include <optional>
#include <sstream>
#include <string>
#include <vector>

#include "array_handlers.h"

namespace molpro::linalg::itsolv {

struct Logger {
  enum Level { None = 0, Trace = 1, Debug = 2, Info = 3, Warn = 4, Error = 5, Fatal = 6 };
  Level max_trace_level = None;  //!< messages at or above Info and at most this level are printed
  Level max_warn_level = Error;
  bool data_dump = false;
  std::ostream* out = &std::cerr;

  void msg(const std::string& message, Level level) const {
    if (level >= Warn) {
      if (level <= max_warn_level && max_trace_level != None) *out << "itsolv " << message << "\n";
      if (level == Fatal) throw std::runtime_error(message);
    } else if (level <= max_trace_level && max_trace_level != None) {
      *out << "itsolv " << message << "\n";
    }
  }
  template <class It>
  void msg(const std::string& prefix, It b, It e, Level level, int precision = 3) const {
    if (!(level <= max_trace_level && max_trace_level != None)) return;
    std::ostringstream s;
    s << prefix << std::setprecision(precision);
    for (; b != e; ++b) s << *b << ", ";
    msg(s.str(), level);
  }
  static std::string scientific(double v) {
    std::ostringstream s;
    s << std::scientific << v;
    return s.str();
  }
};

struct Statistics {
  int iterations = 0;
  int r_creations = 0;
  int q_creations = 0;
  int p_creations = 0;
  int q_deletions = 0;
  int d_creations = 0;
  int best_r_creations = 0;
  int current_r_creations = 0;
  int line_searches = 0;
  int line_search_steps = 0;
  std::string rq_ops, qr_ops, rr_ops, qq_ops, rp_ops, qp_ops;
};

template <typename R, typename Q, typename P>
void read_handler_counts(Statistics& s, ArrayHandlers<R, Q, P>& h) {
  s.rr_ops = h.rr().counter_to_string("R", "R");
  s.qr_ops = h.qr().counter_to_string("Q", "R");
  s.rq_ops = h.rq().counter_to_string("R", "Q");
  s.qq_ops = h.qq().counter_to_string("Q", "Q");
  s.rp_ops = h.rp().counter_to_string("R", "P");
  s.qp_ops = h.qp().counter_to_string("Q", "P");
}

inline std::ostream& operator<<(std::ostream& o, const Statistics& s) {
  if (s.iterations > 0) o << s.iterations << " iterations, ";
  if (s.r_creations > 0) o << s.r_creations << " R vectors, ";
  if (s.q_creations != s.r_creations) o << s.q_creations << " Q creations, ";
  if (s.q_deletions > 0) o << s.q_deletions << " Q deletions, ";
  if (s.p_creations > 0) o << s.p_creations << " P vectors, ";
  if (s.d_creations > 0) o << s.d_creations << " D vectors, ";
  return o << s.rr_ops << " " << s.qr_ops << " " << s.rq_ops << " " << s.qq_ops << " " << s.rp_ops << " " << s.qp_ops;
}

enum class Verbosity { None = 0, Summary = 1, Iteration = 2, Detailed = 3 };

using options_map = std::map<std::string, std::string>;

// "key=value,key=value" -> upper-cased keys (reference itsolv/options_map.h:15, util.cpp:38-56).
inline options_map parse_options(const std::string& s) {
  options_map m;
  std::stringstream ss(s);
  std::string item;
  while (std::getline(ss, item, ',')) {
    auto eq = item.find('=');
    if (eq == std::string::npos) continue;
    auto trim = [](std::string x) {
      x.erase(0, x.find_first_not_of(" \t"));
      x.erase(x.find_last_not_of(" \t") + 1);
      return x;
    };
    std::string key = trim(item.substr(0, eq));
    std::transform(key.begin(), key.end(), key.begin(), [](unsigned char c) { return std::toupper(c); });
    m[key] = trim(item.substr(eq + 1));
  }
  return m;
}

struct Options {
  virtual ~Options() = default;
  Options() = default;
  explicit Options(const options_map& opt) {
    if (opt.count("CONVERGENCE_THRESHOLD")) convergence_threshold = std::stod(opt.at("CONVERGENCE_THRESHOLD"));
    if (opt.count("N_ROOTS")) n_roots = std::stoi(opt.at("N_ROOTS"));
    if (opt.count("MAX_ITER")) max_iter = std::stoi(opt.at("MAX_ITER"));
    if (opt.count("MAX_P")) max_p = std::stod(opt.at("MAX_P"));
    if (opt.count("P_THRESHOLD")) p_threshold = std::stod(opt.at("P_THRESHOLD"));
    if (opt.count("VERBOSITY")) verbosity = Verbosity(std::stoi(opt.at("VERBOSITY")));
  }
  std::optional<double> convergence_threshold;
  std::optional<int> n_roots;
  std::optional<Verbosity> verbosity;
  std::optional<int> max_iter;
  std::optional<double> max_p;
  std::optional<double> p_threshold;
};

struct LinearEigensystemDavidsonOptions : Options {
  LinearEigensystemDavidsonOptions() = default;
  explicit LinearEigensystemDavidsonOptions(const options_map& opt) : Options(opt) {
    if (opt.count("RESET_D")) reset_D = std::stoi(opt.at("RESET_D"));
    if (opt.count("RESET_D_MAX_Q_SIZE")) reset_D_max_Q_size = std::stoi(opt.at("RESET_D_MAX_Q_SIZE"));
    if (opt.count("MAX_SIZE_QSPACE")) max_size_qspace = std::stoi(opt.at("MAX_SIZE_QSPACE"));
    if (opt.count("NORM_THRESH")) norm_thresh = std::stod(opt.at("NORM_THRESH"));
    if (opt.count("SVD_THRESH")) svd_thresh = std::stod(opt.at("SVD_THRESH"));
    if (opt.count("HERMITICITY")) {
      auto v = opt.at("HERMITICITY");
      std::transform(v.begin(), v.end(), v.begin(), [](unsigned char c) { return std::tolower(c); });
      hermiticity = (v == "true" || v == "1" || v == "yes");
    }
    if (opt.count("BLOCK_GRAM_SCHMIDT")) {  // extension, see itsolv_options.block_gram_schmidt
      auto v = opt.at("BLOCK_GRAM_SCHMIDT");
      std::transform(v.begin(), v.end(), v.begin(), [](unsigned char c) { return std::tolower(c); });
      block_gram_schmidt = (v == "true" || v == "1" || v == "yes");
    }
  }
  std::optional<bool> block_gram_schmidt;
  std::optional<int> reset_D;
  std::optional<int> reset_D_max_Q_size;
  std::optional<int> max_size_qspace;
  std::optional<double> norm_thresh;
  std::optional<double> svd_thresh;
  std::optional<bool> hermiticity;
};

struct LinearEquationsDavidsonOptions : LinearEigensystemDavidsonOptions {
  LinearEquationsDavidsonOptions() = default;
  explicit LinearEquationsDavidsonOptions(const options_map& opt) : LinearEigensystemDavidsonOptions(opt) {
    if (opt.count("AUGMENTED_HESSIAN")) augmented_hessian = std::stod(opt.at("AUGMENTED_HESSIAN"));
  }
  std::optional<double> augmented_hessian;
};

struct OptimizeBFGSOptions : Options {
  OptimizeBFGSOptions() = default;
  explicit OptimizeBFGSOptions(const options_map& opt) : Options(opt) {
    auto flag = [](std::string v) {
      std::transform(v.begin(), v.end(), v.begin(), [](unsigned char c) { return std::tolower(c); });
      return v == "true" || v == "1" || v == "yes";
    };
    if (opt.count("MAX_SIZE_QSPACE")) max_size_qspace = std::stoi(opt.at("MAX_SIZE_QSPACE"));
    if (opt.count("STRONG_WOLFE")) strong_Wolfe = flag(opt.at("STRONG_WOLFE"));
    if (opt.count("WOLFE_1")) Wolfe_1 = std::stod(opt.at("WOLFE_1"));
    if (opt.count("WOLFE_2")) Wolfe_2 = std::stod(opt.at("WOLFE_2"));
    if (opt.count("LINESEARCH_TOLERANCE")) linesearch_tolerance = std::stod(opt.at("LINESEARCH_TOLERANCE"));
    if (opt.count("LINESEARCH_GROW_FACTOR")) linesearch_grow_factor = std::stod(opt.at("LINESEARCH_GROW_FACTOR"));
  }
  std::optional<int> max_size_qspace;
  std::optional<bool> strong_Wolfe;
  std::optional<double> Wolfe_1;
  std::optional<double> Wolfe_2;
  std::optional<double> linesearch_tolerance;
  std::optional<double> linesearch_grow_factor;
};

struct NonLinearEquationsDIISOptions : Options {
  NonLinearEquationsDIISOptions() = default;
  explicit NonLinearEquationsDIISOptions(const options_map& opt) : Options(opt) {
    if (opt.count("MAX_SIZE_QSPACE")) max_size_qspace = std::stoi(opt.at("MAX_SIZE_QSPACE"));
    if (opt.count("NORM_THRESH")) norm_thresh = std::stod(opt.at("NORM_THRESH"));
    if (opt.count("SVD_THRESH")) svd_thresh = std::stod(opt.at("SVD_THRESH"));
  }
  std::optional<int> max_size_qspace;
  std::optional<double> norm_thresh;
  std::optional<double> svd_thresh;
};

}  // namespace molpro::linalg::itsolv
