// Solver bookkeeping shared by all layers: Logger levels (reference itsolv/Logger.h:40-69),
// Statistics (reference itsolv/Statistics.h:10-37), Verbosity and Options (reference itsolv/Options.h,
// LinearEigensystemDavidsonOptions.h, NonLinearEquationsDIISOptions.h) with the reference's option
// names parsed from "key=value,key=value" strings, and the string / container utilities of the
// reference's itsolv/util.h:36-120 (StringFacet, capitalize_keys, is_iota, delete_parameters,
// construct_zeroed_copy; implementation util.cpp:1-56).
#pragma once
#include <algorithm>
#include <cctype>
#include <iomanip>
#include <iostream>
#include <iterator>
#include <locale>
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
  // Extension (not in the reference's Statistics): propose_rspace's screening of new R vectors --
  // parameters the redundancy screen removed (propose_rspace.h:481-512) and null norms after the
  // Gram-Schmidt step (:450-465) -- the decisions a near-dependent problem exercises.
  int redundant_params = 0;
  int null_params = 0;
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

namespace util {

//! String helpers of the option parsing (reference itsolv/util.h:104-116, util.cpp:4-56).
class StringFacet {
 public:
  std::string toupper(std::string in) const {
    m_facet.toupper(in.data(), in.data() + in.size());
    return in;
  }
  std::string tolower(std::string in) const {
    m_facet.tolower(in.data(), in.data() + in.size());
    return in;
  }
  //! TRUE / T / 1 and FALSE / F / 0, case- and surrounding-space-insensitive; anything else throws
  bool tobool(const std::string& in) const {
    auto v = toupper(in);
    crop_space(v);
    if (v == "TRUE" || v == "T" || v == "1") return true;
    if (v == "FALSE" || v == "F" || v == "0") return false;
    throw std::runtime_error("value =" + v + ", must be one of {TRUE, T, 1, FALSE, F, 0}");
  }
  //! Strips leading and trailing white space in place.
  static void crop_space(std::string& s) {
    auto not_space = [](unsigned char c) { return !std::isspace(c); };
    s.erase(s.begin(), std::find_if(s.begin(), s.end(), not_space));
    s.erase(std::find_if(s.rbegin(), s.rend(), not_space).base(), s.end());
  }
  //! "k1=v1, k2 : v2; k3=" -> {k1: v1, k2: v2, k3: ""}: fields split at ',' or ';', key from value at
  //! the first '=' or ':', both trimmed; a non-empty field without a separator throws, and parsing
  //! stops at the first empty field ("A=1,,B=2" -> {A: 1}), as reference itsolv/util.cpp:38-56 does.
  static std::map<std::string, std::string> parse_keyval_string(std::string s) {
    std::map<std::string, std::string> out;
    auto trimmed = [](std::string x) {
      crop_space(x);
      return x;
    };
    s += ",;";
    crop_space(s);
    while (!s.empty()) {
      const size_t end = s.find_first_of(",;");
      const std::string field = trimmed(s.substr(0, end));
      if (field.empty()) break;
      const size_t eq = field.find_first_of("=:");
      if (eq == std::string::npos) throw std::runtime_error("String " + field + " cannot be parsed as key,value");
      out[trimmed(field.substr(0, eq))] = trimmed(field.substr(eq + 1));
      s = trimmed(s.substr(end + 1));
    }
    return out;
  }

 private:
  const std::ctype<char>& m_facet = std::use_facet<std::ctype<char>>(std::locale());
};

//! The map with upper-cased keys (reference util.h:30-36).
inline options_map capitalize_keys(const options_map& m, const StringFacet& facet = StringFacet{}) {
  options_map out;
  for (const auto& [k, v] : m) out[facet.toupper(k)] = v;
  return out;
}

//! Whether [first, last) is value_start, value_start + 1, ... (reference util.h:37-46).
template <class ForwardIt, class EndIterator, class Int>
bool is_iota(ForwardIt first, EndIterator last, Int value_start) {
  for (; first != last; ++first, ++value_start)
    if (*first != value_start) return false;
  return true;
}

//! Removes the elements at `indices` from `params` (reference util.h:88-102).
template <class Container>
void delete_parameters(std::vector<int> indices, Container& params) {
  std::sort(indices.begin(), indices.end(), std::greater<int>());
  for (int i : indices) params.erase(std::next(params.begin(), i));
}

//! A copy of `param` of the handler's left type, zeroed (reference util.h:47-53).
template <class Q, class R>
Q construct_zeroed_copy(const R& param, array::ArrayHandler<Q, R>& handler) {
  Q q = handler.copy(param);
  handler.fill(0, q);
  return q;
}

}  // namespace util

// Option string -> map with upper-cased keys: the reference's StringFacet::parse_keyval_string
// followed by the option constructors' capitalize_keys (reference SolverFactory.h:119, Options.cpp:11-12).
inline options_map parse_options(const std::string& s) {
  return util::capitalize_keys(util::StringFacet::parse_keyval_string(s));
}

struct Options {
  virtual ~Options() = default;
  Options() = default;
  explicit Options(const options_map& opt_in) {
    const auto opt = util::capitalize_keys(opt_in);
    if (opt.count("CONVERGENCE_THRESHOLD")) convergence_threshold = std::stod(opt.at("CONVERGENCE_THRESHOLD"));
    if (opt.count("N_ROOTS")) n_roots = std::stoi(opt.at("N_ROOTS"));
    if (opt.count("MAX_ITER")) max_iter = std::stoi(opt.at("MAX_ITER"));
    if (opt.count("MAX_P")) max_p = std::stod(opt.at("MAX_P"));
    if (opt.count("P_THRESHOLD")) p_threshold = std::stod(opt.at("P_THRESHOLD"));
    if (opt.count("VERBOSITY")) verbosity = Verbosity(std::stoi(opt.at("VERBOSITY")));
  }
  //! The base options of `source` (reference Options.cpp:6-9 copies these two).
  void copy(const Options& source) {
    convergence_threshold = source.convergence_threshold;
    n_roots = source.n_roots;
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
  explicit LinearEigensystemDavidsonOptions(const options_map& opt_in) : Options(opt_in) {
    const auto opt = util::capitalize_keys(opt_in);
    const util::StringFacet facet;
    if (opt.count("RESET_D")) reset_D = std::stoi(opt.at("RESET_D"));
    if (opt.count("RESET_D_MAX_Q_SIZE")) reset_D_max_Q_size = std::stoi(opt.at("RESET_D_MAX_Q_SIZE"));
    if (opt.count("MAX_SIZE_QSPACE")) max_size_qspace = std::stoi(opt.at("MAX_SIZE_QSPACE"));
    if (opt.count("NORM_THRESH")) norm_thresh = std::stod(opt.at("NORM_THRESH"));
    if (opt.count("SVD_THRESH")) svd_thresh = std::stod(opt.at("SVD_THRESH"));
    if (opt.count("HERMITICITY")) hermiticity = facet.tobool(opt.at("HERMITICITY"));
    // extension, see itsolv_options.block_gram_schmidt
    if (opt.count("BLOCK_GRAM_SCHMIDT")) block_gram_schmidt = facet.tobool(opt.at("BLOCK_GRAM_SCHMIDT"));
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
  explicit LinearEquationsDavidsonOptions(const options_map& opt_in) : LinearEigensystemDavidsonOptions(opt_in) {
    const auto opt = util::capitalize_keys(opt_in);
    if (opt.count("AUGMENTED_HESSIAN")) augmented_hessian = std::stod(opt.at("AUGMENTED_HESSIAN"));
  }
  std::optional<double> augmented_hessian;
};

struct OptimizeBFGSOptions : Options {
  OptimizeBFGSOptions() = default;
  explicit OptimizeBFGSOptions(const options_map& opt_in) : Options(opt_in) {
    const auto opt = util::capitalize_keys(opt_in);
    const util::StringFacet facet;
    auto flag = [&](const std::string& v) { return facet.tobool(v); };
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
  explicit NonLinearEquationsDIISOptions(const options_map& opt_in) : Options(opt_in) {
    const auto opt = util::capitalize_keys(opt_in);
    if (opt.count("MAX_SIZE_QSPACE")) max_size_qspace = std::stoi(opt.at("MAX_SIZE_QSPACE"));
    if (opt.count("NORM_THRESH")) norm_thresh = std::stod(opt.at("NORM_THRESH"));
    if (opt.count("SVD_THRESH")) svd_thresh = std::stod(opt.at("SVD_THRESH"));
  }
  std::optional<int> max_size_qspace;
  std::optional<double> norm_thresh;
  std::optional<double> svd_thresh;
};

// reference LinearEigensystemRSPTOptions.h / .cpp:6-17: the propose_rspace thresholds
struct LinearEigensystemRSPTOptions : Options {
  LinearEigensystemRSPTOptions() = default;
  explicit LinearEigensystemRSPTOptions(const options_map& opt_in) : Options(opt_in) {
    const auto opt = util::capitalize_keys(opt_in);
    if (opt.count("NORM_THRESH")) norm_thresh = std::stod(opt.at("NORM_THRESH"));
    if (opt.count("SVD_THRESH")) svd_thresh = std::stod(opt.at("SVD_THRESH"));
  }
  std::optional<double> norm_thresh;
  std::optional<double> svd_thresh;
};

// reference OptimizeSDOptions.h: nothing beyond Options
struct OptimizeSDOptions : Options {
  OptimizeSDOptions() = default;
  explicit OptimizeSDOptions(const options_map& opt) : Options(opt) {}
};

}  // namespace molpro::linalg::itsolv
