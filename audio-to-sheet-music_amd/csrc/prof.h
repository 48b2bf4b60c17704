// Live per-kernel timing with HIP events on the launch stream (bench.py's roofline source).
//
// While a context has profiling on (athd_profile_start), forward_impl points t_kprof at the context's KProf and
// every launch wrapper brackets its kernel with an event pair via KScope, tagged with a label equal to the
// kernel's symbol as rocprofv3 prints it (without "void athd::", the argument list and the 'u' suffixes), and
// the ALGORITHMIC work of that launch: flops (MFMA kernels) and bytes (unique operand bytes read + written once).
// With profiling off a KScope costs one thread-local load.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>

namespace athd {

struct KProf {
    std::string only;                      // "" = every kernel, "@section" = every kernel aggregated per forward
                                           // section (KSection), "@sites" = every kernel per call site
                                           // ("kernel@stage.site"), else one kernel label or one call-site label
    struct Rec { std::string label; hipEvent_t a, b; double flops, bytes; };
    struct Agg { std::string label; long long n; double ms, flops, bytes; };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    std::vector<Agg> agg;
    int collect();                         // sync + fold recs into agg (events back to the pool)
    ~KProf();
};

extern thread_local KProf* t_kprof;
extern thread_local const char* t_ksite;    // call-site tags appended as "@stage.site" when ATHD_PROF_SITES=1
extern thread_local const char* t_kstage;
extern thread_local const char* t_ksection;  // "encoder" / "transformer" / "decoder" (profile mode "@section")
struct KSection {
    const char* saved;
    explicit KSection(const char* s) : saved(t_ksection) { t_ksection = s; }
    ~KSection() { t_ksection = saved; }
};
struct KStage {                               // RAII stage tag (e.g. "fenc2", "fdec1")
    const char* saved;
    explicit KStage(const char* s) : saved(t_kstage) { t_kstage = s; }
    ~KStage() { t_kstage = saved; }
};
struct KSite {
    const char* saved;
    explicit KSite(const char* s) : saved(t_ksite) { t_ksite = s; }
    ~KSite() { t_ksite = saved; }
};

class KScope {
  public:
    explicit KScope(hipStream_t s) : s_(s) {}
    bool on() const { return t_kprof != nullptr; }
    void begin(const std::string& label, double flops, double bytes);
    ~KScope();
  private:
    hipStream_t s_;
    int idx_ = -1;
};

}  // namespace athd

#include <cstdarg>
#include <cstdio>
namespace athd {
inline std::string klabel(const char* fmt, ...) {
    char buf[160];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    return buf;
}
}  // namespace athd
