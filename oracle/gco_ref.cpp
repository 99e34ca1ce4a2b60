// gco_ref.cpp -- test harness (oracle side only): drives the reference's own vendored
// Boykov-Kolmogorov max-flow (include/gco-v3.0/energy.h, graph.inl, maxflow.inl, compiled
// from /root/reference, never copied) exactly as GraphCut::labeling does
// (usac/local_optimization/graphcut.cpp:7-101): Energy<float, float, float>, one add_node
// per point, add_term1(i, unary[i], 0) for every point, then add_term2 for each pair in
// order, minimize(), what_segment.  Pins the oracle's BK restatement (orc_bk_label) and the
// product's (usac_host.hpp) -- built into oracle/_ref/ by oracle/Makefile when the reference
// is present.
#include "energy.h"
#include "graph.inl"
#include "maxflow.inl"

extern "C" float gco_ref_label(int n, const float *unary, int m, const int *ei, const int *ej, const float *e00,
                               const float *e01, const float *e10, const float *e11, int *sink_out) {
    typedef Energy<float, float, float> E;
    E *e = new E(n, m, nullptr);
    for (int i = 0; i < n; ++i) e->add_node();
    for (int i = 0; i < n; ++i) e->add_term1(i, unary[i], 0);
    for (int k = 0; k < m; ++k) e->add_term2(ei[k], ej[k], e00[k], e01[k], e10[k], e11[k]);
    const float f = e->minimize();
    for (int i = 0; i < n; ++i) sink_out[i] = e->what_segment(i) == Graph<float, float, float>::SINK;
    delete e;
    return f;
}
