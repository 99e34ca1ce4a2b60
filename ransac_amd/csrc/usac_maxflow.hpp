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
        nd_.reserve(n_nodes);
        arcs_.reserve(2 * n_edges);
    }
    int add_node() {
        nd_.push_back(Node{-1, kNone, -1, 0, 0, 0.f, 0});
        return (int)nd_.size() - 1;
    }
    // graph.h add_tweights
    void add_tweights(int i, float cap_source, float cap_sink) {
        const float delta = nd_[i].tr_cap;
        if (delta > 0) cap_source += delta;
        else cap_sink -= delta;
        flow_ += (cap_source < cap_sink) ? cap_source : cap_sink;
        nd_[i].tr_cap = cap_source - cap_sink;
    }
    // graph.h add_edge
    void add_edge(int i, int j, float cap, float rev_cap) {
        const int a = (int)arcs_.size();
        arcs_.push_back(Arc{j, nd_[i].first, cap});
        nd_[i].first = a;
        arcs_.push_back(Arc{i, nd_[j].first, rev_cap});
        nd_[j].first = a + 1;
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
        const int n = (int)nd_.size();
        for (Node &v : nd_) {
            v.parent = kNone;
            v.next = -1;
            v.ts = 0;
            v.dist = 0;
            v.is_sink = 0;
        }
        q_first_[0] = q_last_[0] = q_first_[1] = q_last_[1] = -1;
        orphan_first_ = orphan_last_ = -1;
        time_ = 0;
        for (int i = 0; i < n; i++) {
            if (nd_[i].tr_cap > 0) {
                nd_[i].is_sink = 0;
                nd_[i].parent = kTerminal;
                set_active(i);
                nd_[i].dist = 1;
            } else if (nd_[i].tr_cap < 0) {
                nd_[i].is_sink = 1;
                nd_[i].parent = kTerminal;
                set_active(i);
                nd_[i].dist = 1;
            }
        }
        int current = -1;
        for (;;) {
            int i = current;
            if (i >= 0) {
                nd_[i].next = -1;
                if (nd_[i].parent == kNone) i = -1;
            }
            if (i < 0 && (i = next_active()) < 0) break;
            int a;
            if (!nd_[i].is_sink) {  // grow the source tree
                for (a = nd_[i].first; a >= 0; a = arcs_[a].next) {
                    if (!arcs_[a].r_cap) continue;
                    const int j = arcs_[a].head;
                    if (nd_[j].parent == kNone) {
                        adopt(j, a ^ 1, i, 0);
                        set_active(j);
                    } else if (nd_[j].is_sink) {
                        break;
                    } else if (nd_[j].ts <= nd_[i].ts && nd_[j].dist > nd_[i].dist) {
                        adopt(j, a ^ 1, i, nd_[j].is_sink);
                    }
                }
            } else {  // grow the sink tree
                for (a = nd_[i].first; a >= 0; a = arcs_[a].next) {
                    if (!arcs_[a ^ 1].r_cap) continue;
                    const int j = arcs_[a].head;
                    if (nd_[j].parent == kNone) {
                        adopt(j, a ^ 1, i, 1);
                        set_active(j);
                    } else if (!nd_[j].is_sink) {
                        a ^= 1;
                        break;
                    } else if (nd_[j].ts <= nd_[i].ts && nd_[j].dist > nd_[i].dist) {
                        adopt(j, a ^ 1, i, nd_[j].is_sink);
                    }
                }
            }
            time_++;
            if (a < 0) {
                current = -1;
                continue;
            }
            nd_[i].next = i;  // stays active
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
                    process_orphan(o, nd_[o].is_sink);
                }
                orphan_first_ = np_next;
            }
        }
        return flow_;
    }
    // what_segment(i) == SINK (free nodes: SOURCE)
    bool is_sink(int i) const { return nd_[i].parent != kNone && nd_[i].is_sink; }

   private:
    static constexpr int kNone = -1, kTerminal = -2, kOrphan = -3, kInfD = 0x7fffffff;

    void adopt(int j, int parent_arc, int i, uint8_t sink) {
        nd_[j].is_sink = sink;
        nd_[j].parent = parent_arc;
        nd_[j].ts = nd_[i].ts;
        nd_[j].dist = nd_[i].dist + 1;
    }
    void set_active(int i) {
        if (nd_[i].next != -1) return;
        if (q_last_[1] >= 0) nd_[q_last_[1]].next = i;
        else q_first_[1] = i;
        q_last_[1] = i;
        nd_[i].next = i;
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
            if (nd_[i].next == i) q_first_[0] = q_last_[0] = -1;
            else q_first_[0] = nd_[i].next;
            nd_[i].next = -1;
            if (nd_[i].parent != kNone) return i;
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
        nd_[i].parent = kOrphan;
        const int np = np_new(i);
        op_next_[np] = orphan_first_;
        orphan_first_ = np;
    }
    void orphan_rear(int i) {
        nd_[i].parent = kOrphan;
        const int np = np_new(i);
        if (orphan_last_ >= 0) op_next_[orphan_last_] = np;
        else orphan_first_ = np;
        orphan_last_ = np;
        op_next_[np] = -1;
    }
    void augment(int mid) {
        int i, a;
        float b = arcs_[mid].r_cap;
        for (i = arcs_[mid ^ 1].head;; i = arcs_[a].head) {
            a = nd_[i].parent;
            if (a == kTerminal) break;
            if (b > arcs_[a ^ 1].r_cap) b = arcs_[a ^ 1].r_cap;
        }
        if (b > nd_[i].tr_cap) b = nd_[i].tr_cap;
        for (i = arcs_[mid].head;; i = arcs_[a].head) {
            a = nd_[i].parent;
            if (a == kTerminal) break;
            if (b > arcs_[a].r_cap) b = arcs_[a].r_cap;
        }
        if (b > -nd_[i].tr_cap) b = -nd_[i].tr_cap;
        arcs_[mid ^ 1].r_cap += b;
        arcs_[mid].r_cap -= b;
        for (i = arcs_[mid ^ 1].head;; i = arcs_[a].head) {
            a = nd_[i].parent;
            if (a == kTerminal) break;
            arcs_[a].r_cap += b;
            arcs_[a ^ 1].r_cap -= b;
            if (!arcs_[a ^ 1].r_cap) orphan_front(i);
        }
        nd_[i].tr_cap -= b;
        if (!nd_[i].tr_cap) orphan_front(i);
        for (i = arcs_[mid].head;; i = arcs_[a].head) {
            a = nd_[i].parent;
            if (a == kTerminal) break;
            arcs_[a ^ 1].r_cap += b;
            arcs_[a].r_cap -= b;
            if (!arcs_[a].r_cap) orphan_front(i);
        }
        nd_[i].tr_cap += b;
        if (!nd_[i].tr_cap) orphan_front(i);
        flow_ += b;
    }
    // process_source_orphan (sink = 0) / process_sink_orphan (sink = 1)
    void process_orphan(int i, uint8_t sink) {
        int a0_min = kNone, d_min = kInfD;
        for (int a0 = nd_[i].first; a0 >= 0; a0 = arcs_[a0].next) {
            if (!(sink ? arcs_[a0].r_cap : arcs_[a0 ^ 1].r_cap)) continue;
            int j = arcs_[a0].head;
            if (nd_[j].is_sink != sink || nd_[j].parent == kNone) continue;
            int d = 0;  // the origin of j
            for (;;) {
                if (nd_[j].ts == time_) {
                    d += nd_[j].dist;
                    break;
                }
                const int a = nd_[j].parent;
                d++;
                if (a == kTerminal) {
                    nd_[j].ts = time_;
                    nd_[j].dist = 1;
                    break;
                }
                if (a == kOrphan) {
                    d = kInfD;
                    break;
                }
                j = arcs_[a].head;
            }
            if (d < kInfD) {
                if (d < d_min) {
                    a0_min = a0;
                    d_min = d;
                }
                for (j = arcs_[a0].head; nd_[j].ts != time_; j = arcs_[nd_[j].parent].head) {
                    nd_[j].ts = time_;
                    nd_[j].dist = d--;
                }
            }
        }
        if ((nd_[i].parent = a0_min) != kNone) {
            nd_[i].ts = time_;
            nd_[i].dist = d_min + 1;
            return;
        }
        for (int a0 = nd_[i].first; a0 >= 0; a0 = arcs_[a0].next) {
            const int j = arcs_[a0].head;
            const int a = nd_[j].parent;
            if (nd_[j].is_sink != sink || a == kNone) continue;
            if (sink ? arcs_[a0].r_cap : arcs_[a0 ^ 1].r_cap) set_active(j);
            if (a != kTerminal && a != kOrphan && arcs_[a].head == i) orphan_rear(j);
        }
    }

    struct Arc {
        int head, next;  // node the arc points to, next arc out of the same node
        float r_cap;     // residual capacity
    };
    struct Node {
        int first, parent, next, ts, dist;  // first out-arc, tree parent arc, active-list link, TIME / DIST
        float tr_cap;                       // > 0: residual SOURCE -> node, < 0: node -> SINK
        uint8_t is_sink;
    };
    std::vector<Arc> arcs_;
    std::vector<Node> nd_;
    std::vector<int> op_node_, op_next_;
    int q_first_[2] = {-1, -1}, q_last_[2] = {-1, -1}, orphan_first_ = -1, orphan_last_ = -1, op_free_ = -1,
        time_ = 0;
    float flow_ = 0.f;
};

}  // namespace usac
