// ORACLE (test infrastructure only): algorithmic FP64 operation count of the dynamics
// restatement.  dyn_oracle.c is compiled a second time as C++ with every `double` replaced by
// `fd`, a trivially-copyable wrapper whose arithmetic operators bump a counter.  The exported
// ABI is unchanged (a one-double standard-layout struct passes exactly like a double), so
// oracle/dyn.py drives this library with the same ctypes signatures.
//
// Counting rule (SURVEY.md §8(d) "FP64 fraction using algorithmic FLOPs/substep counted by an op
// counter in the CPU restatement"): + - * / each count 1 flop; sqrt counts 1 (into both the flop
// and the "special" tally); sin/cos/pow count 1 each into "special" (and 1 flop); comparisons,
// fabs, floor, negation and conversions count 0.  This is the serial algorithm's work: the GPU
// kernel's redundant lanes, symmetrisation copies and address arithmetic are not algorithmic.

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>

static unsigned long long g_flops = 0;
static unsigned long long g_special = 0;

struct fd {
  double v;
  fd() = default;
  template <class T, class = typename std::enable_if<std::is_arithmetic<T>::value>::type>
  constexpr fd(T x) : v((double)x) {}
  explicit operator double() const { return v; }
  explicit operator int() const { return (int)v; }
  explicit operator bool() const { return v != 0.0; }
  fd& operator+=(fd o) { ++g_flops; v += o.v; return *this; }
  fd& operator-=(fd o) { ++g_flops; v -= o.v; return *this; }
  fd& operator*=(fd o) { ++g_flops; v *= o.v; return *this; }
  fd& operator/=(fd o) { ++g_flops; v /= o.v; return *this; }
  fd operator-() const { fd r; r.v = -v; return r; }
  fd operator+() const { return *this; }
};
static_assert(std::is_trivially_copyable<fd>::value && std::is_standard_layout<fd>::value && sizeof(fd) == 8,
              "fd must be ABI-identical to double");

static inline fd mk(double x) { fd r; r.v = x; return r; }
#define RMBX_FD_BINOP(op)                                                                        \
  static inline fd operator op(fd a, fd b) { ++g_flops; return mk(a.v op b.v); }                \
  template <class T, class = typename std::enable_if<std::is_arithmetic<T>::value>::type>      \
  static inline fd operator op(fd a, T b) { ++g_flops; return mk(a.v op (double)b); }           \
  template <class T, class = typename std::enable_if<std::is_arithmetic<T>::value>::type>      \
  static inline fd operator op(T a, fd b) { ++g_flops; return mk((double)a op b.v); }
RMBX_FD_BINOP(+)
RMBX_FD_BINOP(-)
RMBX_FD_BINOP(*)
RMBX_FD_BINOP(/)
#undef RMBX_FD_BINOP
#define RMBX_FD_CMP(op)                                                                          \
  static inline bool operator op(fd a, fd b) { return a.v op b.v; }                             \
  template <class T, class = typename std::enable_if<std::is_arithmetic<T>::value>::type>      \
  static inline bool operator op(fd a, T b) { return a.v op (double)b; }                        \
  template <class T, class = typename std::enable_if<std::is_arithmetic<T>::value>::type>      \
  static inline bool operator op(T a, fd b) { return (double)a op b.v; }
RMBX_FD_CMP(<)
RMBX_FD_CMP(>)
RMBX_FD_CMP(<=)
RMBX_FD_CMP(>=)
RMBX_FD_CMP(==)
RMBX_FD_CMP(!=)
#undef RMBX_FD_CMP
static inline bool operator!(fd a) { return a.v == 0.0; }

static inline fd sqrt(fd a) { ++g_flops; ++g_special; return mk(std::sqrt(a.v)); }
static inline fd sin(fd a) { ++g_flops; ++g_special; return mk(std::sin(a.v)); }
static inline fd cos(fd a) { ++g_flops; ++g_special; return mk(std::cos(a.v)); }
static inline fd pow(fd a, fd b) { ++g_flops; ++g_special; return mk(std::pow(a.v, b.v)); }
static inline fd fabs(fd a) { return mk(std::fabs(a.v)); }
static inline fd floor(fd a) { return mk(std::floor(a.v)); }
static inline bool isfinite(fd a) { return std::isfinite(a.v); }

#define double fd
extern "C" {
#include "dyn_oracle.c"
}
#undef double

extern "C" unsigned long long orc_flops(void) { return g_flops; }
extern "C" unsigned long long orc_special_ops(void) { return g_special; }
extern "C" void orc_flops_reset(void) { g_flops = 0; g_special = 0; }
