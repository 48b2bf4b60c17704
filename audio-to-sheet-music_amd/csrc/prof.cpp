#include "prof.h"

#include <cstdlib>
#include <map>

namespace athd {

thread_local KProf* t_kprof = nullptr;
thread_local const char* t_ksite = nullptr;
thread_local const char* t_kstage = nullptr;
thread_local const char* t_ksection = nullptr;

static bool sites_on() {
    static const bool on = [] {
        const char* e = std::getenv("ATHD_PROF_SITES");
        return e && *e && *e != '0';
    }();
    return on;
}

void KScope::begin(const std::string& label0, double flops, double bytes) {
    KProf* p = t_kprof;
    if (!p) return;
    // call-site label "kernel@stage.site" (when the launch has a stage / site tag)
    std::string site = label0;
    if (t_kstage || t_ksite) {
        site += "@";
        if (t_kstage) site += t_kstage;
        if (t_kstage && t_ksite) site += ".";
        if (t_ksite) site += t_ksite;
    }
    std::string label = label0;
    if (p->only == "@section") {
        label = t_ksection ? t_ksection : "other";
    } else if (p->only == "@sites" || sites_on()) {
        label = site;
    }
    if (!p->only.empty() && p->only[0] != '@') {
        // one kernel ("gemm5_kernel<129>") or one call site of it ("gemm5_kernel<129>@transformer.linear1")
        if (p->only != (p->only.find('@') != std::string::npos ? site : label0)) return;
        label = p->only;
    }
    hipEvent_t ev[2];
    for (auto& e : ev) {
        if (!p->pool.empty()) {
            e = p->pool.back();
            p->pool.pop_back();
        } else if (hipEventCreate(&e) != hipSuccess) {
            return;
        }
    }
    if (hipEventRecord(ev[0], s_) != hipSuccess) return;
    idx_ = (int)p->recs.size();
    p->recs.push_back({label, ev[0], ev[1], flops, bytes});
}

KScope::~KScope() {
    if (idx_ >= 0 && t_kprof) (void)hipEventRecord(t_kprof->recs[idx_].b, s_);
}

int KProf::collect() {
    std::map<std::string, size_t> at;
    for (size_t i = 0; i < agg.size(); ++i) at[agg[i].label] = i;
    int rc = 0;
    for (auto& r : recs) {
        float ms = 0.f;
        if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) rc = -1;
        auto it = at.find(r.label);
        if (it == at.end()) {
            at[r.label] = agg.size();
            agg.push_back({r.label, 0, 0.0, 0.0, 0.0});
            it = at.find(r.label);
        }
        Agg& g = agg[it->second];
        g.n += 1;
        g.ms += ms;
        g.flops += r.flops;
        g.bytes += r.bytes;
        pool.push_back(r.a);
        pool.push_back(r.b);
    }
    recs.clear();
    return rc;
}

KProf::~KProf() {
    for (auto& r : recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    for (auto e : pool) (void)hipEventDestroy(e);
}

}  // namespace athd
