// usac_maxflow.hpp -- Boykov-Kolmogorov min-cut for the graph-cut LO (GraphCut::labeling,
// graphcut.cpp:7-101), with the reference's energy encoding (include/gco-v3.0/energy.h) and
// the exact search-tree discipline of its vendored max-flow (gco-v3.0 graph.h, maxflow.inl):
// arcs in pairs (sister = a ^ 1) prepended to their tail's list, two FIFO queues of active
// nodes, augmentation orphans pushed to the front of the orphan list and adoption orphans to
// the rear, the TIME / DIST origin heuristic, float capacities in gco's operation order.
// With float capacities the final trees depend on that order, so it is kept; the labels
// (what_segment == SINK) are then the reference's (pinned in tests against the gco sources
// built into oracle/_ref).  Host code: max-flow is a sequential augmenting-path algorithm;
// the residuals it is built from come from the device.
#pragma once
#include <stdint.h>

#include <vector>

namespace usac {

class BkGraph {
   public:
    BkGraph(int n_nodes, size_t n_edges) {
        first_.reserve(n_nodes);
        tr_cap_.reserve(n_nodes);
        head_.reserve(2 * n_edges);
        anext_.reserve(2 * n_edges);
        r_cap_.reserve(2 * n_edges);
    }
    int add_node() {
        first_.push_back(-1);
        tr_cap_.push_back(0.f);
        return (int)first_.size() - 1;
    }
    // graph.h add_tweights
    void add_tweights(int i, float cap_source, float cap_sink) {
        const float delta = tr_cap_[i];
        if (delta > 0) cap_source += delta;
        else cap_sink -= delta;
        flow_ += (cap_source < cap_sink) ? cap_source : cap_sink;
        tr_cap_[i] = cap_source - cap_sink;
    }
    // graph.h add_edge
    void add_edge(int i, int j, float cap, float rev_cap) {
        const int a = (int)head_.size();
        head_.push_back(j);
        anext_.push_back(first_[i]);
        r_cap_.push_back(cap);
        first_[i] = a;
        head_.push_back(i);
        anext_.push_back(first_[j]);
        r_cap_.push_back(rev_cap);
        first_[j] = a + 1;
    }
    // energy.h add_term1(x, E0, E1) / add_term2(x, y, E00, E01, E10, E11)
    void add_term1(int x, float e0, float e1) { add_tweights(x, e1, e0); }
    void add_term2(int x, int y, float A, float B, float C, float D) {
        add_tweights(x, D, A);
        B -= A;
        C -= D;
        if (B < 0) {
            add_tweights(x, 0, B);
            add_tweights(y, 0, -B);
            add_edge(x, y, 0, B + C);
        } else if (C < 0) {
            add_tweights(x, 0, -C);
            add_tweights(y, 0, C);
            add_edge(x, y, B + C, 0);
        } else {
            add_edge(x, y, B, C);
        }
    }

    // Graph::maxflow(reuse_trees = false)
    float maxflow() {
        const int n = (int)first_.size();
        parent_.assign(n, kNone);
        next_.assign(n, -1);
        ts_.assign(n, 0);
        dist_.assign(n, 0);
        is_sink_.assign(n, 0);
        q_first_[0] = q_last_[0] = q_first_[1] = q_last_[1] = -1;
        orphan_first_ = orphan_last_ = -1;
        time_ = 0;
        for (int i = 0; i < n; i++) {
            if (tr_cap_[i] > 0) {
                is_sink_[i] = 0;
                parent_[i] = kTerminal;
                set_active(i);
                dist_[i] = 1;
            } else if (tr_cap_[i] < 0) {
                is_sink_[i] = 1;
                parent_[i] = kTerminal;
                set_active(i);
                dist_[i] = 1;
            }
        }
        int current = -1;
        for (;;) {
            int i = current;
            if (i >= 0) {
                next_[i] = -1;
                if (parent_[i] == kNone) i = -1;
            }
            if (i < 0 && (i = next_active()) < 0) break;
            int a;
            if (!is_sink_[i]) {  // grow the source tree
                for (a = first_[i]; a >= 0; a = anext_[a]) {
                    if (!r_cap_[a]) continue;
                    const int j = head_[a];
                    if (parent_[j] == kNone) {
                        adopt(j, a ^ 1, i, 0);
                        set_active(j);
                    } else if (is_sink_[j]) {
                        break;
                    } else if (ts_[j] <= ts_[i] && dist_[j] > dist_[i]) {
                        adopt(j, a ^ 1, i, is_sink_[j]);
                    }
                }
            } else {  // grow the sink tree
                for (a = first_[i]; a >= 0; a = anext_[a]) {
                    if (!r_cap_[a ^ 1]) continue;
                    const int j = head_[a];
                    if (parent_[j] == kNone) {
                        adopt(j, a ^ 1, i, 1);
                        set_active(j);
                    } else if (!is_sink_[j]) {
                        a ^= 1;
                        break;
                    } else if (ts_[j] <= ts_[i] && dist_[j] > dist_[i]) {
                        adopt(j, a ^ 1, i, is_sink_[j]);
                    }
                }
            }
            time_++;
            if (a < 0) {
                current = -1;
                continue;
            }
            next_[i] = i;  // stays active
            current = i;
            augment(a);
            int np;
            while ((np = orphan_first_) >= 0) {  // adoption
                const int np_next = op_next_[np];
                op_next_[np] = -1;
                while ((np = orphan_first_) >= 0) {
                    orphan_first_ = op_next_[np];
                    const int o = op_node_[np];
                    op_next_[np] = op_free_;  // back to the pool
                    op_free_ = np;
                    if (orphan_first_ < 0) orphan_last_ = -1;
                    process_orphan(o, is_sink_[o]);
                }
                orphan_first_ = np_next;
            }
        }
        return flow_;
    }
    // what_segment(i) == SINK (free nodes: SOURCE)
    bool is_sink(int i) const { return parent_[i] != kNone && is_sink_[i]; }

   private:
    static constexpr int kNone = -1, kTerminal = -2, kOrphan = -3, kInfD = 0x7fffffff;

    void adopt(int j, int parent_arc, int i, uint8_t sink) {
        is_sink_[j] = sink;
        parent_[j] = parent_arc;
        ts_[j] = ts_[i];
        dist_[j] = dist_[i] + 1;
    }
    void set_active(int i) {
        if (next_[i] != -1) return;
        if (q_last_[1] >= 0) next_[q_last_[1]] = i;
        else q_first_[1] = i;
        q_last_[1] = i;
        next_[i] = i;
    }
    int next_active() {
        for (;;) {
            int i = q_first_[0];
            if (i < 0) {
                q_first_[0] = i = q_first_[1];
                q_last_[0] = q_last_[1];
                q_first_[1] = q_last_[1] = -1;
                if (i < 0) return -1;
            }
            if (next_[i] == i) q_first_[0] = q_last_[0] = -1;
            else q_first_[0] = next_[i];
            next_[i] = -1;
            if (parent_[i] != kNone) return i;
        }
    }
    int np_new(int node) {
        int np;
        if (op_free_ >= 0) {
            np = op_free_;
            op_free_ = op_next_[np];
            op_node_[np] = node;
        } else {
            np = (int)op_node_.size();
            op_node_.push_back(node);
            op_next_.push_back(-1);
        }
        return np;
    }
    void orphan_front(int i) {
        parent_[i] = kOrphan;
        const int np = np_new(i);
        op_next_[np] = orphan_first_;
        orphan_first_ = np;
    }
    void orphan_rear(int i) {
        parent_[i] = kOrphan;
        const int np = np_new(i);
        if (orphan_last_ >= 0) op_next_[orphan_last_] = np;
        else orphan_first_ = np;
        orphan_last_ = np;
        op_next_[np] = -1;
    }
    void augment(int mid) {
        int i, a;
        float b = r_cap_[mid];
        for (i = head_[mid ^ 1];; i = head_[a]) {
            a = parent_[i];
            if (a == kTerminal) break;
            if (b > r_cap_[a ^ 1]) b = r_cap_[a ^ 1];
        }
        if (b > tr_cap_[i]) b = tr_cap_[i];
        for (i = head_[mid];; i = head_[a]) {
            a = parent_[i];
            if (a == kTerminal) break;
            if (b > r_cap_[a]) b = r_cap_[a];
        }
        if (b > -tr_cap_[i]) b = -tr_cap_[i];
        r_cap_[mid ^ 1] += b;
        r_cap_[mid] -= b;
        for (i = head_[mid ^ 1];; i = head_[a]) {
            a = parent_[i];
            if (a == kTerminal) break;
            r_cap_[a] += b;
            r_cap_[a ^ 1] -= b;
            if (!r_cap_[a ^ 1]) orphan_front(i);
        }
        tr_cap_[i] -= b;
        if (!tr_cap_[i]) orphan_front(i);
        for (i = head_[mid];; i = head_[a]) {
            a = parent_[i];
            if (a == kTerminal) break;
            r_cap_[a ^ 1] += b;
            r_cap_[a] -= b;
            if (!r_cap_[a]) orphan_front(i);
        }
        tr_cap_[i] += b;
        if (!tr_cap_[i]) orphan_front(i);
        flow_ += b;
    }
    // process_source_orphan (sink = 0) / process_sink_orphan (sink = 1)
    void process_orphan(int i, uint8_t sink) {
        int a0_min = kNone, d_min = kInfD;
        for (int a0 = first_[i]; a0 >= 0; a0 = anext_[a0]) {
            if (!(sink ? r_cap_[a0] : r_cap_[a0 ^ 1])) continue;
            int j = head_[a0];
            if (is_sink_[j] != sink || parent_[j] == kNone) continue;
            int d = 0;  // the origin of j
            for (;;) {
                if (ts_[j] == time_) {
                    d += dist_[j];
                    break;
                }
                const int a = parent_[j];
                d++;
                if (a == kTerminal) {
                    ts_[j] = time_;
                    dist_[j] = 1;
                    break;
                }
                if (a == kOrphan) {
                    d = kInfD;
                    break;
                }
                j = head_[a];
            }
            if (d < kInfD) {
                if (d < d_min) {
                    a0_min = a0;
                    d_min = d;
                }
                for (j = head_[a0]; ts_[j] != time_; j = head_[parent_[j]]) {
                    ts_[j] = time_;
                    dist_[j] = d--;
                }
            }
        }
        if ((parent_[i] = a0_min) != kNone) {
            ts_[i] = time_;
            dist_[i] = d_min + 1;
            return;
        }
        for (int a0 = first_[i]; a0 >= 0; a0 = anext_[a0]) {
            const int j = head_[a0];
            const int a = parent_[j];
            if (is_sink_[j] != sink || a == kNone) continue;
            if (sink ? r_cap_[a0] : r_cap_[a0 ^ 1]) set_active(j);
            if (a != kTerminal && a != kOrphan && head_[a] == i) orphan_rear(j);
        }
    }

    std::vector<int> first_, head_, anext_, parent_, next_, ts_, dist_, op_node_, op_next_;
    std::vector<float> tr_cap_, r_cap_;
    std::vector<uint8_t> is_sink_;
    int q_first_[2] = {-1, -1}, q_last_[2] = {-1, -1}, orphan_first_ = -1, orphan_last_ = -1, op_free_ = -1,
        time_ = 0;
    float flow_ = 0.f;
};

}  // namespace usac
