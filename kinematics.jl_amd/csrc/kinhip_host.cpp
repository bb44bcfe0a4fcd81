// kinhip_host.cpp -- C-ABI of libkinhip.so: models (Mechanism trees), plan
// staging (tree -> device program, kinhip_prog.h) and launches.
//
// Reference semantics restated here (host side):
//   Mechanism / create_rptable / is_relevant   src/mechanism.jl:117-181, 277
//   joint_transform (static parts, fp64)       src/mechanism.jl:90-103
//   set_joint_angles column layout             src/mechanism.jl:223-231
//   get_jacobian! column relevance / errors    src/algorithm.jl:83-106
//   add_new_link                                src/mechanism.jl:238-267
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <condition_variable>
#include <sstream>
#include <string>
#include <type_traits>
#include <vector>

#include "kinhip.h"
#include "kinhip_host.h"
#include "kinhip_internal.h"

namespace kinhip {

static thread_local std::string g_err;

int set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

namespace {

// rigid 3x4, row-major rotation
struct M34 {
    double r[9];
    double t[3];
};

M34 m_identity() {
    M34 m{};
    m.r[0] = m.r[4] = m.r[8] = 1.0;
    return m;
}

bool m_is_identity(const M34& m) {
    const M34 I = m_identity();
    return memcmp(&m, &I, sizeof(M34)) == 0;
}

M34 m_mul(const M34& a, const M34& b) {
    M34 c;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j)
            c.r[3 * i + j] = a.r[3 * i] * b.r[j] + a.r[3 * i + 1] * b.r[3 + j] + a.r[3 * i + 2] * b.r[6 + j];
        c.t[i] = a.r[3 * i] * b.t[0] + a.r[3 * i + 1] * b.t[1] + a.r[3 * i + 2] * b.t[2] + a.t[i];
    }
    return c;
}

M34 m_from_col16(const double* T) {
    M34 m;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) m.r[3 * i + j] = T[i + 4 * j];
        m.t[i] = T[i + 12];
    }
    return m;
}

M34 m_rigid_inverse(const M34& a) {  // [R t]^-1 = [R^T  -R^T t]
    M34 m{};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) m.r[3 * i + j] = a.r[3 * j + i];
    for (int i = 0; i < 3; ++i) m.t[i] = -(m.r[3 * i] * a.t[0] + m.r[3 * i + 1] * a.t[1] + m.r[3 * i + 2] * a.t[2]);
    return m;
}

M34 m_rot_transpose(const M34& a) {  // inverse of a pure rotation
    M34 m{};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) m.r[3 * i + j] = a.r[3 * j + i];
    return m;
}

// Rotations.jl UnitQuaternion(w, x, y, z) (normalising) -> RotMatrix
M34 m_quat(double w, double x, double y, double z) {
    const double n = sqrt(w * w + x * x + y * y + z * z);
    w /= n; x /= n; y /= n; z /= n;
    const double ww = w * w, xx = x * x, yy = y * y, zz = z * z;
    const double xy = x * y, zw = w * z, xz = x * z, yw = y * w, yz = y * z, xw = w * x;
    M34 m{};
    m.r[0] = ww + xx - yy - zz; m.r[1] = 2 * (xy - zw);     m.r[2] = 2 * (xz + yw);
    m.r[3] = 2 * (xy + zw);     m.r[4] = ww - xx + yy - zz; m.r[5] = 2 * (yz - xw);
    m.r[6] = 2 * (xz - yw);     m.r[7] = 2 * (yz + xw);     m.r[8] = ww - xx - yy + zz;
    return m;
}

template <typename T>
void to_row12(const M34& m, T* out) {
    for (int i = 0; i < 3; ++i) {
        out[4 * i + 0] = (T)m.r[3 * i + 0];
        out[4 * i + 1] = (T)m.r[3 * i + 1];
        out[4 * i + 2] = (T)m.r[3 * i + 2];
        out[4 * i + 3] = (T)m.t[i];
    }
}

}  // namespace
}  // namespace kinhip

using namespace kinhip;

struct kin_plan;

struct kin_model {
    int32_t n_links = 0;
    std::vector<int32_t> jtype, jplink, jclink;  // 1-based link ids
    std::vector<double> jpose;                    // [J][16] column-major
    std::vector<double> jaxis;                    // [J][3]
    std::vector<double> jlo, jhi;
    std::vector<int32_t> link_pjoint;               // 0-based joint, -1 root
    std::vector<std::vector<int32_t>> child_joints;  // per link, 0-based joints in joint order
    std::vector<double> angles;                      // m.angles
    bool with_base = false;
    uint64_t version = 0;
    std::mutex mu;
    std::map<std::string, kin_plan*> cache;

    int32_t n_joints() const { return (int32_t)jtype.size(); }
    int32_t plink(int32_t l) const { return link_pjoint[l] < 0 ? -1 : jplink[link_pjoint[l]] - 1; }
    M34 pose(int32_t j) const { return m_from_col16(&jpose[16 * j]); }
    // joint motion at a constant angle (the right factor of joint_transform)
    M34 motion_at(int32_t j, double a) const {
        if (jtype[j] == KIN_JOINT_FIXED || a == 0.0) return m_identity();
        const double* ax = &jaxis[3 * j];
        if (jtype[j] == KIN_JOINT_REVOLUTE) {
            const double s = sin(0.5 * a), c = cos(0.5 * a);
            return m_quat(c, ax[0] * s, ax[1] * s, ax[2] * s);
        }
        M34 m = m_identity();
        m.t[0] = ax[0] * a; m.t[1] = ax[1] * a; m.t[2] = ax[2] * a;
        return m;
    }
    // joint_transform(joint, angle), src/mechanism.jl:90-103
    M34 joint_tf(int32_t j, double a) const {
        if (jtype[j] == KIN_JOINT_FIXED || a == 0.0) return pose(j);
        return m_mul(pose(j), motion_at(j, a));
    }
    bool relevant(int32_t j, int32_t l) const {  // rptable[j][l]: l in subtree of j's child
        const int32_t c = jclink[j] - 1;
        for (int32_t x = l, guard = 0; x >= 0 && guard <= n_links; x = plink(x), ++guard)
            if (x == c) return true;
        return false;
    }
};

struct kin_sdf {
    int device = -1;        // HIP device holding the box tables (current device at creation)
    // boxes attached to a scene mechanism (kin_sdf_create_attached): group table + scene steps
    bool attached = false;
    int32_t n_groups = 0, scene_cols = 0, scene_base_col = -1;
    void* d_scene_f32 = nullptr;  // KSceneGroup[n_groups], then KSceneStep<float>[] at scene_steps_off
    void* d_scene_f64 = nullptr;
    size_t scene_steps_off = 0;
    int32_t n_boxes = 0;
    int32_t n_aabb = 0;     // the first n_aabb boxes are axis-aligned (KAabb table after the KBox array)
    double bc[3] = {0, 0, 0}, bh[3] = {0, 0, 0};  // world-aligned box enclosing every box (broad phase, coll_body)
    void* d_f32 = nullptr;
    void* d_f64 = nullptr;
    // host copies of an attached union's tables (kin_plan_specialize_scene compiles them in), and an id that
    // is never reused (the plans' scene-specialised kernels are keyed by it)
    uint64_t uid = 0;
    std::vector<KSceneGroup> h_groups;
    std::vector<KSceneStep<float>> h_ssf;
    std::vector<KSceneStep<double>> h_ssd;
    std::vector<KBox<float>> h_bf;
    std::vector<KBox<double>> h_bd;
    std::vector<KAabb<float>> h_af;
    std::vector<KAabb<double>> h_ad;
    ~kin_sdf() {
        if (d_f32) (void)hipFree(d_f32);
        if (d_f64) (void)hipFree(d_f64);
        if (d_scene_f32) (void)hipFree(d_scene_f32);
        if (d_scene_f64) (void)hipFree(d_scene_f64);
    }
};

struct kin_plan {
    int device = -1;  // HIP device holding the staged program (current device at creation); runs must match
    int32_t dtype = KIN_F32;
    int32_t nqcols = 0, rows = 0, ncols = 0, n_q = 0, n_out = 0;
    bool has_jac = false, with_base = false, has_rpy = false;
    bool ik_ok = false;
    int32_t out_link0 = 0, jac_link = 0;  // first output link / Jacobian link (kin_pose_const_batch)
    std::string ik_why;
    void* d_steps = nullptr;
    KProg<float> pf{};
    KProg<double> pd{};
    LaunchGeom geom{256, 0, 8};
    // collision plans (kin_coll_plan_create); is_coll_ik: also an IK plan of the spheres' chain
    // (kin_coll_ik_plan_create: kin_ik_dls_batch, kin_ik_coll_batch, kin_coll_batch)
    bool is_coll = false;
    bool is_coll_ik = false;
    int32_t n_sph = 0;
    void* d_sph = nullptr;
    // spheres on several chains: one staged program per chain (kin_coll_plan_create)
    std::vector<std::unique_ptr<kin_plan>> parts;
    // host copy of the staged program (plan specialisation, kinhip_jit.cpp)
    std::vector<unsigned char> h_steps, h_sph;
    int32_t n_steps = 0;
    JitKernels* jit = nullptr;
    uint32_t jit_mask = 0;
    // two-phase IK schedule scratch (launch_ik_dls): allocated by the first kin_ik_dls_batch call that
    // runs the two-phase schedule.  An eager call takes an eager set (0..kIkEagerSets-1) and is ordered
    // after the set's previous call: by stream order when that call ran on the same stream (one handle
    // other than hipStreamPerThread names one stream for every thread), else through the set's event --
    // nothing to wait for once it has completed, otherwise a host wait (hipEventSynchronize; see
    // ik_dls_batch for why not hipStreamWaitEvent).  No guess about which stream or thread a set belongs
    // to is needed, so any thread, stream or handle may take any set.  The choice only affects
    // concurrency: the set this stream used last, else one whose last call has finished, else the least
    // recently used one.  ik_busy covers the host window between taking a set and recording its event; a
    // call that finds all sets in that window waits for one (ik_cv).  A call made inside a stream capture
    // takes one of the remaining sets for good (the captured graph replays with it, so it never meets an
    // eager call or another graph), and once those are gone further captures run the one-phase schedule.
    static constexpr int kIkScratchSets = 8;
    static constexpr int kIkEagerSets = 4;
    static constexpr int64_t kIkScratchCap = int64_t(1) << 20;
    mutable std::mutex ik_mu;
    mutable std::condition_variable ik_cv;
    mutable void* d_ikscr = nullptr;
    mutable int ik_captured = 0;  // sets kIkEagerSets .. kIkEagerSets + ik_captured - 1 belong to graphs
    mutable hipEvent_t ik_ev[kIkEagerSets] = {};   // recorded after a set's last call (null: unused)
    mutable void* ik_stream[kIkEagerSets] = {};    // stream handle of that call
    mutable uint64_t ik_tick[kIkEagerSets] = {};   // when that call took the set (least recently used)
    mutable bool ik_busy[kIkEagerSets] = {};       // a host thread is launching into the set
    mutable uint64_t ik_ticks = 0;
    mutable kin_ik_sched_stats ik_stats{};         // kin_plan_ik_sched_stats (tests)
    // collision-aware IK program (kin_coll_ik_plan_create, k_ik_tree): the needed tree, host copies
    // (plan specialisation) and one device allocation [KIkcStep<T> steps | KSphere<T> spheres]
    KIkcProg<float> ikf{};
    KIkcProg<double> ikd{};
    std::vector<unsigned char> h_ikc_steps, h_ikc_sph;
    void* d_ikc = nullptr;
    size_t ikc_sph_off = 0;
    // kin_plan_specialize_scene: k_coll_scene kernels with one attached union compiled in, by kin_sdf uid
    mutable std::mutex scene_mu;
    std::map<uint64_t, JitKernels*> scene_jit;
    const JitFns* scene_fns(uint64_t uid) const {
        std::lock_guard<std::mutex> lk(scene_mu);
        const auto it = scene_jit.find(uid);
        return it == scene_jit.end() ? nullptr : jit_fns(it->second);
    }
    ~kin_plan() {
        for (auto& kv : scene_jit) jit_destroy(kv.second);
        if (d_ikc) (void)hipFree(d_ikc);
        for (hipEvent_t e : ik_ev)
            if (e) (void)hipEventDestroy(e);
        if (d_ikscr) (void)hipFree(d_ikscr);
        jit_destroy(jit);
        if (d_steps) (void)hipFree(d_steps);
        if (d_sph) (void)hipFree(d_sph);
    }
};

namespace {

int validate_tree(const kin_tree_desc* d) {
    if (!d) return set_error(KIN_E_INVALID, "kin_model_create: null desc");
    if (d->n_links < 1 || d->n_joints < 0) return set_error(KIN_E_INVALID, "kin_model_create: bad sizes");
    if (d->n_joints > 0 && (!d->joint_type || !d->joint_plink || !d->joint_clink || !d->joint_pose || !d->joint_axis))
        return set_error(KIN_E_INVALID, "kin_model_create: null joint arrays");
    std::vector<int> parents(d->n_links, 0);
    for (int32_t j = 0; j < d->n_joints; ++j) {
        const int32_t t = d->joint_type[j];
        if (t != KIN_JOINT_FIXED && t != KIN_JOINT_REVOLUTE && t != KIN_JOINT_PRISMATIC)
            return set_error(KIN_E_INVALID, "kin_model_create: joint " + std::to_string(j + 1) + " has unknown type");
        const int32_t p = d->joint_plink[j], c = d->joint_clink[j];
        if (p < 1 || p > d->n_links || c < 1 || c > d->n_links)
            return set_error(KIN_E_KEY, "kin_model_create: joint " + std::to_string(j + 1) + " link id out of range");
        if (++parents[c - 1] > 1)
            return set_error(KIN_E_INVALID, "kin_model_create: link " + std::to_string(c) + " has two parent joints");
    }
    return KIN_OK;
}

int finish_model(kin_model* m) {
    const int32_t L = m->n_links, J = m->n_joints();
    m->link_pjoint.assign(L, -1);
    m->child_joints.assign(L, {});
    for (int32_t j = 0; j < J; ++j) {
        m->link_pjoint[m->jclink[j] - 1] = j;
        m->child_joints[m->jplink[j] - 1].push_back(j);
    }
    for (int32_t l = 0; l < L; ++l) {  // cycle check
        int32_t x = l, guard = 0;
        while (x >= 0) {
            if (++guard > L + 1) return set_error(KIN_E_INVALID, "kin_model_create: the joint graph has a cycle");
            x = m->plink(x);
        }
    }
    return KIN_OK;
}

// rotation A with A e_z = unit axis (exact for signed basis axes)
M34 align_z(const double* a, double* scale) {
    const double n = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    *scale = n;
    if (n == 0.0) return m_identity();
    const double z[3] = {a[0] / n, a[1] / n, a[2] / n};
    if (z[0] == 0.0 && z[1] == 0.0 && z[2] == 1.0) return m_identity();
    double h[3] = {0, 0, 1};
    if (fabs(z[2]) >= 0.9) { h[0] = 1; h[2] = 0; }
    double u[3] = {h[1] * z[2] - h[2] * z[1], h[2] * z[0] - h[0] * z[2], h[0] * z[1] - h[1] * z[0]};
    const double un = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    for (double& v : u) v /= un;
    const double v[3] = {z[1] * u[2] - z[2] * u[1], z[2] * u[0] - z[0] * u[2], z[0] * u[1] - z[1] * u[0]};
    M34 A{};
    for (int i = 0; i < 3; ++i) {
        A.r[3 * i + 0] = u[i];
        A.r[3 * i + 1] = v[i];
        A.r[3 * i + 2] = z[i];
    }
    return A;
}

struct SD {  // staged step, fp64
    M34 F, X;
    bool hasX = false;
    double scale = 1, lo = -INFINITY, hi = INFINITY;
    int32_t kind = MOT_NONE, jkind = MOT_NONE, qcol = -1, flags = 0, out = -1, load = LOAD_NONE, save = -1;
    int32_t sph0 = 0, sph1 = 0;
    uint64_t colmask = 0;
};

struct SphD {  // staged collision sphere
    int32_t step;  // phase-A step whose frame carries it (-1: root frame)
    double c[3];   // centre in that (canonical) frame
    double r;
    int32_t out;
};

struct Stager {
    const kin_model& m;
    const kin_plan_desc& d;
    std::vector<int32_t> qcol;
    std::vector<char> moving, rec, needed, node;
    std::vector<uint64_t> colmask;
    std::vector<std::vector<int32_t>> outs_of, cchildren;  // per link
    std::vector<M34> Xinv;
    std::vector<char> hasX;
    std::vector<SD> steps;
    uint64_t zmask = 0;
    std::vector<int32_t> chain, chain_step;  // phase-A nodes root..spine and their edge steps (-1: none)
    // collision plans
    const kin_coll_desc* coll = nullptr;
    const int32_t* sph_out = nullptr;  // global sphere index of each desc sphere (multi-chain plans)
    std::vector<SphD> spheres;
    int32_t sph_root0 = 0, sph_root1 = 0;
    // a static last edge into the spine folded into Xlast (no step): the spine link and the
    // transform from the previous chain node's canonical frame to it (spheres on the spine, k_ik_coll)
    int32_t fold_spine = -1;
    M34 fold_X = m_identity();
    // LDS slots
    std::vector<int> slot_of_link, slot_refs;
    std::vector<int> free_slots;
    int n_slots = 0;

    Stager(const kin_model& m_, const kin_plan_desc& d_) : m(m_), d(d_) {}

    int alloc_slot() {
        if (!free_slots.empty()) {
            int s = free_slots.back();
            free_slots.pop_back();
            return s;
        }
        slot_refs.push_back(0);
        return n_slots++;
    }
    void consume(int slot) {
        if (slot >= 0 && --slot_refs[slot] == 0) free_slots.push_back(slot);
    }

    int32_t cparent(int32_t v) const {  // nearest node ancestor (compressed parent), -1 for roots
        for (int32_t x = m.plink(v); x >= 0; x = m.plink(x))
            if (node[x]) return x;
        return -1;
    }

    // edge u -> v (v a node); appends the edge step and duplicate-output steps
    void emit_edge(int32_t v, int32_t load) {
        SD st;
        st.load = load;
        std::vector<int32_t> path;  // joints from cparent(v) down to v
        for (int32_t x = v; x >= 0 && !(x != v && node[x]); x = m.plink(x))
            if (m.link_pjoint[x] >= 0) path.push_back(m.link_pjoint[x]);
        const int32_t u = cparent(v);
        if (u < 0 || path.empty()) {  // v is a root: pseudo-step on the root frame
            st.F = m_identity();
            Xinv[v] = m_identity();
            hasX[v] = 0;
        } else {
            M34 S = hasX[u] ? Xinv[u] : m_identity();
            for (size_t k = path.size() - 1; k >= 1; --k) S = m_mul(S, m.joint_tf(path[k], m.angles[path[k]]));
            const int32_t jm = path[0];
            if (moving[jm] || rec[jm]) {
                double scale;
                const M34 A = align_z(&m.jaxis[3 * jm], &scale);
                st.F = m_mul(m_mul(S, m.pose(jm)), A);
                st.scale = scale;
                st.jkind = m.jtype[jm] == KIN_JOINT_PRISMATIC ? MOT_PRISM : MOT_REV;
                st.lo = m.jlo[jm];
                st.hi = m.jhi[jm];
                if (rec[jm]) {
                    st.flags |= SF_REC;
                    st.colmask = colmask[jm];
                }
                if (moving[jm]) {
                    st.kind = st.jkind;
                    st.qcol = qcol[jm];
                    if (st.kind == MOT_REV && scale != 1.0) st.flags |= SF_SCALE;
                    Xinv[v] = m_rot_transpose(A);
                } else {
                    Xinv[v] = m_mul(m_rot_transpose(A), m.motion_at(jm, m.angles[jm]));
                }
                hasX[v] = !m_is_identity(Xinv[v]);
            } else {
                st.F = m_mul(S, m.joint_tf(jm, m.angles[jm]));
                Xinv[v] = m_identity();
                hasX[v] = 0;
            }
        }
        st.X = Xinv[v];
        st.hasX = hasX[v];
        if (st.hasX) st.flags |= SF_HAS_X;
        const auto& o = outs_of[v];
        st.out = o.empty() ? -1 : o[0];
        steps.push_back(st);
        for (size_t k = 1; k < o.size(); ++k) {  // same link requested again: identity pseudo-steps
            SD dup;
            dup.F = m_identity();
            dup.X = st.X;
            dup.hasX = st.hasX;
            dup.flags = st.hasX ? SF_HAS_X : 0;
            dup.out = o[k];
            steps.push_back(dup);
        }
    }

    void emit_subtree(int32_t v, int32_t load) {
        emit_edge(v, load);
        const size_t edge_step = steps.size() - 1 - (outs_of[v].size() > 1 ? outs_of[v].size() - 1 : 0);
        const auto& ch = cchildren[v];
        if (ch.empty()) return;
        int slot = -1;
        if (ch.size() >= 2) {
            slot = alloc_slot();
            slot_refs[slot] = (int)ch.size() - 1;
            steps[edge_step].save = slot;
        }
        emit_subtree(ch[0], LOAD_NONE);
        for (size_t k = 1; k < ch.size(); ++k) {
            emit_subtree_loaded(ch[k], slot);
        }
    }
    void emit_subtree_loaded(int32_t v, int slot) {
        emit_subtree(v, slot);
        consume(slot);
    }

    // spheres = links (src/collision.jl:39-49), each carried by the nearest chain node above it;
    // the static path from that node (and the node's canonical-frame correction) is folded into
    // the centre, in fp64
    int stage_spheres(int32_t sroot) {
        const int32_t L = m.n_links;
        std::vector<int32_t> on_chain(L, -1);
        for (size_t k = 0; k < chain.size(); ++k) on_chain[chain[k]] = (int32_t)k;
        for (int32_t k = 0; k < coll->n_spheres; ++k) {
            const int32_t lk = coll->sphere_link_ids[k] - 1;
            if (lk < 0 || lk >= L) return set_error(KIN_E_KEY, "coll plan: sphere link id out of range");
            std::vector<int32_t> path;
            int32_t x = lk;
            while (x >= 0 && on_chain[x] < 0) {
                const int32_t j = m.link_pjoint[x];
                if (j < 0) break;
                if (moving[j])
                    return set_error(KIN_E_UNSUPPORTED, "coll plan: sphere " + std::to_string(k) +
                                                            " hangs off a moving joint outside the chain");
                path.push_back(j);
                x = m.plink(x);
            }
            if (x < 0 || on_chain[x] < 0)
                return set_error(KIN_E_UNSUPPORTED, "coll plan: sphere " + std::to_string(k) + " is on another tree");
            M34 S = hasX[x] ? Xinv[x] : m_identity();
            if (x == fold_spine) {  // the spine has no step: carry the sphere by the node above it
                S = fold_X;
                x = chain[on_chain[x] - 1];
            }
            for (size_t pi = path.size(); pi-- > 0;) S = m_mul(S, m.joint_tf(path[pi], m.angles[path[pi]]));
            SphD sd;
            const double c0 = coll->centers ? coll->centers[3 * k] : 0.0;
            const double c1 = coll->centers ? coll->centers[3 * k + 1] : 0.0;
            const double c2 = coll->centers ? coll->centers[3 * k + 2] : 0.0;
            for (int i = 0; i < 3; ++i) sd.c[i] = S.r[3 * i] * c0 + S.r[3 * i + 1] * c1 + S.r[3 * i + 2] * c2 + S.t[i];
            sd.r = coll->radii[k];
            sd.out = sph_out ? sph_out[k] : k;
            sd.step = (x == sroot) ? -1 : chain_step[on_chain[x]];
            if (x != sroot && sd.step < 0) return set_error(KIN_E_INVALID, "coll plan: internal (no step)");
            spheres.push_back(sd);
        }
        std::stable_sort(spheres.begin(), spheres.end(), [](const SphD& a, const SphD& b) { return a.step < b.step; });
        for (size_t k = 0; k < spheres.size(); ++k) {
            const int32_t st = spheres[k].step;
            if (st < 0) {
                sph_root1 = (int32_t)k + 1;
            } else {
                if (steps[st].sph1 == 0) steps[st].sph0 = (int32_t)k;
                steps[st].sph1 = (int32_t)k + 1;
            }
        }
        return KIN_OK;
    }

    int run(kin_plan& P) {
        const int32_t L = m.n_links, J = m.n_joints();
        if (d.dtype != KIN_F32 && d.dtype != KIN_F64) return set_error(KIN_E_INVALID, "plan: bad dtype");
        if (d.n_q < 0 || d.n_out < 0 || d.n_jac < 0) return set_error(KIN_E_INVALID, "plan: negative count");
        if ((d.n_q && !d.q_joint_ids) || (d.n_out && !d.out_link_ids) || (d.n_jac && !d.jac_joint_ids))
            return set_error(KIN_E_INVALID, "plan: null id array");
        qcol.assign(J, -1);
        for (int32_t c = 0; c < d.n_q; ++c) {
            const int32_t j = d.q_joint_ids[c] - 1;
            if (j < 0 || j >= J) return set_error(KIN_E_KEY, "plan: q joint id " + std::to_string(j + 1) + " out of range");
            qcol[j] = c;  // set_joint_angles: a repeated joint keeps the last value
        }
        moving.assign(J, 0);
        for (int32_t j = 0; j < J; ++j) moving[j] = qcol[j] >= 0 && m.jtype[j] != KIN_JOINT_FIXED;
        rec.assign(J, 0);
        colmask.assign(J, 0);
        const int32_t jl = d.jac_link_id - 1;
        const bool has_jac = d.jac_link_id != 0;
        if (has_jac) {
            if (jl < 0 || jl >= L) return set_error(KIN_E_KEY, "plan: jac link id out of range");
            if (d.n_jac > kMaxJacCols)
                return set_error(KIN_E_UNSUPPORTED, "plan: more than 64 Jacobian columns");
            for (int32_t c = 0; c < d.n_jac; ++c) {
                const int32_t j = d.jac_joint_ids[c] - 1;
                if (j < 0 || j >= J) return set_error(KIN_E_KEY, "plan: jac joint id out of range");
                if (m.relevant(j, jl)) {
                    if (m.jtype[j] == KIN_JOINT_FIXED)
                        return set_error(KIN_E_METHOD, "MethodError: no joint_jacobian! method for fixed joint " +
                                                           std::to_string(j + 1));
                    rec[j] = 1;
                    colmask[j] |= 1ull << c;
                } else {
                    zmask |= 1ull << c;
                }
            }
        } else if (d.n_jac) {
            return set_error(KIN_E_INVALID, "plan: Jacobian joints without a Jacobian link");
        }
        outs_of.assign(L, {});
        for (int32_t o = 0; o < d.n_out; ++o) {
            const int32_t l = d.out_link_ids[o] - 1;
            if (l < 0 || l >= L) return set_error(KIN_E_KEY, "plan: output link id out of range");
            outs_of[l].push_back(o);
        }
        needed.assign(L, 0);
        auto mark = [&](int32_t l) {
            for (int32_t x = l; x >= 0 && !needed[x]; x = m.plink(x)) needed[x] = 1;
        };
        for (int32_t o = 0; o < d.n_out; ++o) mark(d.out_link_ids[o] - 1);
        if (has_jac) mark(jl);
        // spine = the chain evaluated straight-line in registers (phase A): the
        // Jacobian link, else the needed link with the most moving joints above it
        int32_t spine = has_jac ? jl : -1;
        if (!has_jac) {
            int best = -1, best_depth = -1;
            for (int32_t o = 0; o < d.n_out; ++o) {
                const int32_t l = d.out_link_ids[o] - 1;
                int mv = 0, depth = 0;
                for (int32_t x = l; m.link_pjoint[x] >= 0; x = m.plink(x)) {
                    mv += moving[m.link_pjoint[x]];
                    ++depth;
                }
                if (mv > best || (mv == best && depth > best_depth)) {
                    best = mv;
                    best_depth = depth;
                    spine = l;
                }
            }
        }
        // nodes: links whose frame is materialised (roots, children of moving or
        // recorded joints, outputs, the spine); static branch points are folded
        node.assign(L, 0);
        for (int32_t l = 0; l < L; ++l) {
            if (!needed[l]) continue;
            const int32_t pj = m.link_pjoint[l];
            node[l] = pj < 0 || moving[pj] || rec[pj] || !outs_of[l].empty() || l == spine;
        }
        // compressed children in tree (joint) order
        cchildren.assign(L, {});
        std::vector<int32_t> roots;
        for (int32_t l = 0; l < L; ++l)
            if (needed[l] && m.link_pjoint[l] < 0) roots.push_back(l);
        for (int32_t r : roots) {
            std::vector<std::pair<int32_t, int32_t>> work{{r, -1}};  // (link, nearest node ancestor)
            while (!work.empty()) {
                auto [x, anc] = work.back();
                work.pop_back();
                if (node[x] && anc >= 0) cchildren[anc].push_back(x);
                const int32_t a2 = node[x] ? x : anc;
                const auto& cj = m.child_joints[x];
                for (auto it = cj.rbegin(); it != cj.rend(); ++it) {
                    const int32_t c = m.jclink[*it] - 1;
                    if (needed[c]) work.push_back({c, a2});
                }
            }
        }
        Xinv.assign(L, m_identity());
        hasX.assign(L, 0);

        // ---- phase A: root -> spine, straight-line, no loads ----
        std::vector<std::pair<int32_t, int32_t>> pending;  // (child node, parent node)
        int32_t sroot = -1;
        int32_t nA = 0, spine_out = -1;
        M34 Xl = m_identity();
        int32_t lhx = 0;
        slot_of_link.assign(L, -1);
        if (spine >= 0) {
            chain.clear();  // nodes root..spine
            for (int32_t x = spine; x >= 0; x = cparent(x)) chain.push_back(x);
            std::reverse(chain.begin(), chain.end());
            sroot = chain[0];
            const size_t K = chain.size() - 1;
            // a static last edge into a leaf spine folds into Xlast (no step)
            bool fold = false;
            if (K >= 1 && cchildren[spine].empty() && outs_of[spine].size() <= 1) {
                const int32_t pj = m.link_pjoint[spine];
                fold = !(moving[pj] || rec[pj]);
            }
            std::vector<int32_t> edge_step(chain.size(), -1);
            for (size_t k = 0; k < chain.size(); ++k) {
                const int32_t v = chain[k];
                if (k == K && fold) {
                    const int32_t u = chain[k - 1];
                    Xl = hasX[u] ? Xinv[u] : m_identity();
                    std::vector<int32_t> path;
                    for (int32_t x = v; x != u; x = m.plink(x)) path.push_back(m.link_pjoint[x]);
                    for (size_t p = path.size(); p-- > 0;) Xl = m_mul(Xl, m.joint_tf(path[p], m.angles[path[p]]));
                    lhx = !m_is_identity(Xl);
                    spine_out = outs_of[v].empty() ? -1 : outs_of[v][0];
                    fold_spine = v;
                    fold_X = Xl;
                } else if (k > 0 || !outs_of[v].empty()) {
                    edge_step[k] = (int32_t)steps.size();
                    emit_edge(v, LOAD_NONE);
                }
                const int32_t next = k < K ? chain[k + 1] : -1;
                for (int32_t c : cchildren[v])
                    if (c != next) pending.push_back({c, v});
            }
            if (!fold) {
                Xl = Xinv[spine];
                lhx = hasX[spine];
            }
            chain_step = edge_step;
            nA = (int32_t)steps.size();
            if (nA > kMaxChain)
                return set_error(KIN_E_UNSUPPORTED, "plan: root -> spine chain has " + std::to_string(nA) +
                                                        " steps (max " + std::to_string(kMaxChain) + ")");
            // slots for chain nodes with pending children (the root frame needs none)
            std::map<int32_t, int> cnt;
            for (auto& pc : pending) cnt[pc.second]++;
            for (size_t k = 0; k < chain.size(); ++k) {
                const int32_t v = chain[k];
                auto it = cnt.find(v);
                if (it == cnt.end() || v == sroot) continue;
                const int s = alloc_slot();
                slot_refs[s] = it->second;
                slot_of_link[v] = s;
                steps[edge_step[k]].save = s;
            }
            // pad to the compiled chain bound with identity steps
            const int32_t bound = pick_chain_bound(nA);
            while ((int32_t)steps.size() < bound) {
                SD pad;
                pad.F = m_identity();
                pad.X = m_identity();
                pad.scale = 0.0;
                steps.push_back(pad);
            }
            nA = bound;
        }
        if (coll) {
            const int rc = stage_spheres(sroot);
            if (rc != KIN_OK) return rc;
        }
        // ---- phase B ----
        for (auto& pc : pending) {
            const int32_t v = pc.first, u = pc.second;
            if (u == sroot) {
                emit_subtree(v, LOAD_ROOT);
            } else {
                const int s = slot_of_link[u];
                emit_subtree(v, s);
                consume(s);
            }
        }
        for (int32_t r : roots) {
            if (r == sroot) continue;
            if (!outs_of[r].empty()) emit_edge(r, LOAD_ROOT);
            for (int32_t c : cchildren[r]) emit_subtree(c, LOAD_ROOT);
        }
        if (n_slots > kMaxSlots)
            return set_error(KIN_E_UNSUPPORTED, "plan: needs " + std::to_string(n_slots) + " LDS branch slots (max 8)");

        // ---- finalize ----
        P.dtype = d.dtype;
        P.with_base = m.with_base;
        P.n_q = d.n_q;
        P.n_out = d.n_out;
        P.nqcols = d.n_q + (m.with_base ? 3 : 0);
        P.has_jac = has_jac;
        P.rows = (d.jac_flags & KIN_WITH_ROT) ? 6 : 3;
        P.ncols = has_jac ? d.n_jac + (m.with_base ? 3 : 0) : 0;
        P.has_rpy = (d.jac_flags & KIN_RPY_JAC) != 0;
        P.out_link0 = d.n_out > 0 ? d.out_link_ids[0] : 0;
        P.jac_link = has_jac ? d.jac_link_id : 0;
        int32_t pflags = 0;
        if (has_jac) pflags |= PF_JAC;
        if (d.jac_flags & KIN_WITH_ROT) pflags |= PF_WITH_ROT;
        if (d.jac_flags & KIN_RPY_JAC) pflags |= PF_RPY;
        if (d.jac_flags & KIN_ZERO_FILL) pflags |= PF_ZERO;
        if (m.with_base) pflags |= PF_BASE;
        const size_t esz = d.dtype == KIN_F32 ? sizeof(float) : sizeof(double);
        int block = 256;
        while (block > 64 && (size_t)n_slots * 12 * block * esz > 64 * 1024) block /= 2;
        P.geom.block = block;
        P.geom.lds = (size_t)n_slots * 12 * block * esz;  // per-lane branch slots
        P.geom.maxA = nA;
        auto fill = [&](auto& K, auto* host) {
            using T = std::remove_reference_t<decltype(host[0].F[0])>;
            K.nA = nA;
            K.nS = (int32_t)steps.size();
            K.n_slots = n_slots;
            K.rows = P.rows;
            K.n_jac = d.n_jac;
            K.flags = pflags;
            K.base_col = d.n_q;
            K.last_has_x = lhx;
            K.spine_out = spine_out;
            K.zmask = zmask;
            K.n_sph = (int32_t)spheres.size();
            K.sph_root0 = sph_root0;
            K.sph_root1 = sph_root1;
            to_row12<T>(Xl, K.Xlast);
            for (size_t s = 0; s < steps.size(); ++s) {
                const SD& a = steps[s];
                auto& b = host[s];
                memset(&b, 0, sizeof(b));
                to_row12<T>(a.F, b.F);
                to_row12<T>(a.X, b.X);
                b.scale = (T)a.scale;
                b.lo = (T)a.lo;
                b.hi = (T)a.hi;
                b.kind = a.kind;
                b.jkind = a.jkind;
                b.qcol = a.qcol;
                b.flags = a.flags;
                b.out = a.out;
                b.load = a.load;
                b.save = a.save;
                b.sph0 = a.sph0;
                b.sph1 = a.sph1;
                b.colmask = a.colmask;
            }
        };
        size_t bytes;
        std::vector<unsigned char> host;
        if (d.dtype == KIN_F32) {
            bytes = std::max<size_t>(1, steps.size()) * sizeof(KStep<float>);
            host.assign(bytes, 0);
            fill(P.pf, reinterpret_cast<KStep<float>*>(host.data()));
        } else {
            bytes = std::max<size_t>(1, steps.size()) * sizeof(KStep<double>);
            host.assign(bytes, 0);
            fill(P.pd, reinterpret_cast<KStep<double>*>(host.data()));
        }
        P.h_steps = host;
        P.n_steps = (int32_t)steps.size();
        hipError_t e = hipGetDevice(&P.device);
        if (e != hipSuccess) return set_error(KIN_E_DEVICE, std::string("hipGetDevice: ") + hipGetErrorString(e));
        e = hipMalloc(&P.d_steps, bytes);
        if (e != hipSuccess) {
            P.d_steps = nullptr;
            return set_error(KIN_E_DEVICE, std::string("hipMalloc: ") + hipGetErrorString(e));
        }
        e = hipMemcpy(P.d_steps, host.data(), bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) return set_error(KIN_E_DEVICE, std::string("hipMemcpy: ") + hipGetErrorString(e));
        if (coll) {
            P.is_coll = true;
            P.n_sph = (int32_t)spheres.size();
            auto put = [&](auto* tag) -> int {
                using TS = std::remove_pointer_t<decltype(tag)>;
                std::vector<TS> hs(std::max<size_t>(1, spheres.size()));
                memset(hs.data(), 0, sizeof(TS) * hs.size());
                for (size_t k = 0; k < spheres.size(); ++k) {
                    for (int i = 0; i < 3; ++i) hs[k].c[i] = spheres[k].c[i];
                    hs[k].r = spheres[k].r;
                    hs[k].out = spheres[k].out;
                }
                const size_t nb = sizeof(TS) * hs.size();
                P.h_sph.assign((const unsigned char*)hs.data(), (const unsigned char*)hs.data() + nb);
                hipError_t e2 = hipMalloc(&P.d_sph, nb);
                if (e2 != hipSuccess) {
                    P.d_sph = nullptr;
                    return set_error(KIN_E_DEVICE, std::string("hipMalloc: ") + hipGetErrorString(e2));
                }
                e2 = hipMemcpy(P.d_sph, hs.data(), nb, hipMemcpyHostToDevice);
                if (e2 != hipSuccess) return set_error(KIN_E_DEVICE, std::string("hipMemcpy: ") + hipGetErrorString(e2));
                return KIN_OK;
            };
            const int rc = d.dtype == KIN_F32 ? put((KSphere<float>*)nullptr) : put((KSphere<double>*)nullptr);
            if (rc != KIN_OK) return rc;
        }

        // IK eligibility: Jacobian joints == q joints (same order, no repeats), no rpy rows
        P.ik_ok = has_jac && d.n_jac == d.n_q && !(d.jac_flags & KIN_RPY_JAC);
        if (P.ik_ok) {
            std::vector<char> seen(J, 0);
            for (int32_t c = 0; c < d.n_q; ++c) {
                if (d.q_joint_ids[c] != d.jac_joint_ids[c]) { P.ik_ok = false; P.ik_why = "jac joints != q joints"; }
                if (seen[d.q_joint_ids[c] - 1]++) { P.ik_ok = false; P.ik_why = "repeated joint"; }
            }
        } else {
            P.ik_why = "IK needs a Jacobian over the q joints without rpy rows";
        }
        return KIN_OK;
    }
};

int plan_create(const kin_model* m, const kin_plan_desc* d, kin_plan** out) {
    if (!m || !d || !out) return set_error(KIN_E_INVALID, "kin_plan_create: null argument");
    auto P = std::make_unique<kin_plan>();
    Stager s(*m, *d);
    const int rc = s.run(*P);
    if (rc != KIN_OK) return rc;
    *out = P.release();
    return KIN_OK;
}

bool dev_ptr_ok(const void* p) { return p != nullptr; }

// A plan's program (and its specialised module) lives on the device that was current when it was
// created; launching it from another device would read that memory through the wrong context.
int check_device(int owner, const char* fn, const char* what) {
    int cur = -1;
    const hipError_t e = hipGetDevice(&cur);
    if (e != hipSuccess) return set_error(KIN_E_DEVICE, std::string(fn) + ": hipGetDevice: " + hipGetErrorString(e));
    if (cur != owner)
        return set_error(KIN_E_INVALID, std::string(fn) + ": " + what + " lives on HIP device " + std::to_string(owner) +
                                            " but the current device is " + std::to_string(cur));
    return KIN_OK;
}

std::string cache_key(const kin_model* m, const kin_plan_desc& d) {
    std::ostringstream k;
    int dev = -1;
    (void)hipGetDevice(&dev);  // one cached plan per device (kin_get_*_batch from several devices)
    k << dev << '#' << m->version << '|' << d.dtype << '|' << d.jac_link_id << '|' << d.jac_flags << "|q";
    for (int32_t c = 0; c < d.n_q; ++c) k << ',' << d.q_joint_ids[c];
    k << "|o";
    for (int32_t c = 0; c < d.n_out; ++c) k << ',' << d.out_link_ids[c];
    k << "|j";
    for (int32_t c = 0; c < d.n_jac; ++c) k << ',' << d.jac_joint_ids[c];
    return k.str();
}

int cached_plan(kin_model* m, const kin_plan_desc& d, kin_plan** out) {
    const std::string key = cache_key(m, d);
    std::lock_guard<std::mutex> g(m->mu);
    auto it = m->cache.find(key);
    if (it != m->cache.end()) {
        *out = it->second;
        return KIN_OK;
    }
    kin_plan* p = nullptr;
    const int rc = plan_create(m, &d, &p);
    if (rc != KIN_OK) return rc;
    m->cache[key] = p;
    *out = p;
    return KIN_OK;
}

void clear_cache(kin_model* m) {
    std::lock_guard<std::mutex> g(m->mu);
    for (auto& kv : m->cache) delete kv.second;
    m->cache.clear();
}

}  // namespace

namespace {
// Signed axis permutation test for a box rotation (columns of R = box axes in
// the world).  perm[i] = world axis of box axis i.
bool axis_permutation(const double* pose16, int perm[3]) {
    int used = 0;
    for (int i = 0; i < 3; ++i) {
        perm[i] = -1;
        for (int j = 0; j < 3; ++j) {
            const double a = std::fabs(pose16[4 * i + j]);  // column-major: R[j][i]
            if (a > 1e-12 && std::fabs(a - 1.0) > 1e-12) return false;
            if (a > 0.5) {
                if (perm[i] >= 0) return false;
                perm[i] = j;
            }
        }
        if (perm[i] < 0 || (used & (1 << perm[i]))) return false;
        used |= 1 << perm[i];
    }
    return true;
}

template <typename T>
hipError_t upload_boxes(void** dst, const std::vector<KBox<T>>& b, const std::vector<KAabb<T>>& a) {
    const size_t nb = sizeof(KBox<T>) * b.size(), na = sizeof(KAabb<T>) * a.size();
    hipError_t e = hipMalloc(dst, nb + na);
    if (e == hipSuccess) e = hipMemcpy(*dst, b.data(), nb, hipMemcpyHostToDevice);
    if (e == hipSuccess && na) e = hipMemcpy((char*)*dst + nb, a.data(), na, hipMemcpyHostToDevice);
    return e;
}
}  // namespace

extern "C" {

int kin_abi_version(void) { return KINHIP_ABI_VERSION; }

const char* kin_last_error(void) { return g_err.c_str(); }

int kin_limits(int32_t* max_chain, int32_t* max_jac_cols, int32_t* max_slots) {
    if (max_chain) *max_chain = kMaxChain;
    if (max_jac_cols) *max_jac_cols = kMaxJacCols;
    if (max_slots) *max_slots = kMaxSlots;
    return KIN_OK;
}

int kin_model_create(const kin_tree_desc* d, kin_model** out) {
    if (!out) return set_error(KIN_E_INVALID, "kin_model_create: null out");
    int rc = validate_tree(d);
    if (rc != KIN_OK) return rc;
    auto m = std::make_unique<kin_model>();
    const int32_t J = d->n_joints;
    m->n_links = d->n_links;
    m->jtype.assign(d->joint_type, d->joint_type + J);
    m->jplink.assign(d->joint_plink, d->joint_plink + J);
    m->jclink.assign(d->joint_clink, d->joint_clink + J);
    m->jpose.assign(d->joint_pose, d->joint_pose + 16 * (size_t)J);
    m->jaxis.assign(d->joint_axis, d->joint_axis + 3 * (size_t)J);
    m->jlo.resize(J);
    m->jhi.resize(J);
    for (int32_t j = 0; j < J; ++j) {
        m->jlo[j] = d->joint_lower ? d->joint_lower[j] : -INFINITY;
        m->jhi[j] = d->joint_upper ? d->joint_upper[j] : INFINITY;
    }
    m->angles.assign(J, 0.0);
    m->with_base = d->with_base != 0;
    rc = finish_model(m.get());
    if (rc != KIN_OK) return rc;
    *out = m.release();
    return KIN_OK;
}

int kin_model_destroy(kin_model* m) {
    if (!m) return KIN_OK;
    clear_cache(m);
    delete m;
    return KIN_OK;
}

int kin_model_num_links(const kin_model* m, int32_t* out) {
    if (!m || !out) return set_error(KIN_E_INVALID, "null argument");
    *out = m->n_links;
    return KIN_OK;
}

int kin_model_num_joints(const kin_model* m, int32_t* out) {
    if (!m || !out) return set_error(KIN_E_INVALID, "null argument");
    *out = m->n_joints();
    return KIN_OK;
}

int kin_model_set_angles(kin_model* m, const double* angles) {
    if (!m) return set_error(KIN_E_INVALID, "null model");
    if (angles) m->angles.assign(angles, angles + m->n_joints());
    else m->angles.assign(m->n_joints(), 0.0);
    clear_cache(m);
    m->version++;
    return KIN_OK;
}

int kin_model_is_relevant(const kin_model* m, int32_t joint_id, int32_t link_id, int32_t* out) {
    if (!m || !out) return set_error(KIN_E_INVALID, "null argument");
    if (joint_id < 1 || joint_id > m->n_joints()) return set_error(KIN_E_KEY, "joint id out of range");
    if (link_id < 1 || link_id > m->n_links) return set_error(KIN_E_KEY, "link id out of range");
    *out = m->relevant(joint_id - 1, link_id - 1) ? 1 : 0;
    return KIN_OK;
}

int kin_model_add_link(kin_model* m, int32_t parent, const double* pose16, int32_t* new_id) {
    if (!m || !pose16) return set_error(KIN_E_INVALID, "null argument");
    if (parent < 1 || parent > m->n_links) return set_error(KIN_E_KEY, "parent link id out of range");
    m->n_links += 1;
    m->jtype.push_back(KIN_JOINT_FIXED);
    m->jplink.push_back(parent);
    m->jclink.push_back(m->n_links);
    m->jpose.insert(m->jpose.end(), pose16, pose16 + 16);
    const double ax[3] = {1, 0, 0};
    m->jaxis.insert(m->jaxis.end(), ax, ax + 3);
    m->jlo.push_back(-INFINITY);
    m->jhi.push_back(INFINITY);
    m->angles.push_back(0.0);
    const int rc = finish_model(m);
    if (rc != KIN_OK) return rc;
    clear_cache(m);
    m->version++;
    if (new_id) *new_id = m->n_links;
    return KIN_OK;
}

int kin_plan_create(const kin_model* m, const kin_plan_desc* d, kin_plan** out) { return plan_create(m, d, out); }

int kin_plan_destroy(kin_plan* p) {
    delete p;
    return KIN_OK;
}

int kin_plan_shape(const kin_plan* p, int32_t* nq, int32_t* rows, int32_t* cols) {
    if (!p) return set_error(KIN_E_INVALID, "null plan");
    if (nq) *nq = p->nqcols;
    if (rows) *rows = p->has_jac ? p->rows : 0;
    if (cols) *cols = p->ncols;
    return KIN_OK;
}

namespace {
int plan_run(const kin_plan* p, const void* q, int64_t ldq, int64_t n, void* poses, int64_t ldp, void* jac,
             int64_t ldj, const TileArgs& ta, void* stream, const char* fn) {
    auto bad = [&](const char* what) { return set_error(KIN_E_INVALID, std::string(fn) + ": " + what); };
    if (!p) return bad("null plan");
    if (n < 0) return bad("n < 0");
    if (n == 0) return KIN_OK;
    if (const int rc = check_device(p->device, fn, "the plan")) return rc;
    const int64_t span = std::min(ta.tile, n);  // configurations along one row of one tile
    if (p->nqcols > 0 && (!dev_ptr_ok(q) || ldq < span)) return bad("bad q / ldq");
    if (p->n_out > 0 && !poses) return bad("null poses");
    if (poses && ldp < span) return bad("ldp < tile");
    if (p->has_jac && (!jac || ldj < span)) return bad("bad jac / ldj");
    hipError_t e;
    if (p->dtype == KIN_F32)
        e = launch_fk<float>(p->pf, (const KStep<float>*)p->d_steps, p->geom, (const float*)q, ldq, n, (float*)poses,
                             ldp, (float*)jac, ldj, ta, jit_fns(p->jit),
                             (hipStream_t)stream);
    else
        e = launch_fk<double>(p->pd, (const KStep<double>*)p->d_steps, p->geom, (const double*)q, ldq, n,
                              (double*)poses, ldp, (double*)jac, ldj, ta,
                              jit_fns(p->jit), (hipStream_t)stream);
    if (e != hipSuccess) return set_error(KIN_E_DEVICE, std::string("k_fk launch: ") + hipGetErrorString(e));
    return KIN_OK;
}
}  // namespace

int kin_plan_run(const kin_plan* p, const void* q, int64_t ldq, int64_t n, void* poses, int64_t ldp, void* jac,
                 int64_t ldj, void* stream) {
    return plan_run(p, q, ldq, n, poses, ldp, jac, ldj, plain_soa(n), stream, "kin_plan_run");
}

int kin_plan_run_tiled(const kin_plan* p, int64_t tile, const void* q, int64_t ldq, int64_t tsq, int64_t n,
                       void* poses, int64_t ldp, int64_t tsp, void* jac, int64_t ldj, int64_t tsj, void* stream) {
    auto bad = [&](const char* what) { return set_error(KIN_E_INVALID, std::string("kin_plan_run_tiled: ") + what); };
    if (!p) return bad("null plan");
    if (tile < 256 || tile % 256 != 0 || tile > (int64_t(1) << 26)) return bad("tile must be a multiple of 256 <= 2^26");
    if (n > tile) {  // several tiles: their strides must not overlap a tile's rows
        if (p->nqcols > 0 && tsq < (int64_t)p->nqcols * ldq) return bad("tsq < n_qcols * ldq");
        if (p->n_out > 0 && tsp < (int64_t)p->n_out * 12 * ldp) return bad("tsp < n_out * 12 * ldp");
        if (p->has_jac && tsj < (int64_t)p->ncols * p->rows * ldj) return bad("tsj < cols * rows * ldj");
    }
    return plan_run(p, q, ldq, n, poses, ldp, jac, ldj, TileArgs{tile, tsq, tsp, tsj}, stream, "kin_plan_run_tiled");
}

namespace {
int specialize_one(kin_plan* p, uint32_t kernels) {
    if ((p->jit_mask & kernels) == kernels) return KIN_OK;
    kernels |= p->jit_mask;
    JitKernels* k = nullptr;
    const bool ikc = p->is_coll_ik;
    const int rc = p->dtype == KIN_F32
                       ? jit_build<float>(p->pf, (const KStep<float>*)p->h_steps.data(), p->n_steps, p->geom.maxA,
                                          p->h_sph.empty() ? nullptr : p->h_sph.data(), p->n_sph, ikc ? &p->ikf : nullptr,
                                          p->h_ikc_steps.data(), p->h_ikc_sph.data(), kernels, &k)
                       : jit_build<double>(p->pd, (const KStep<double>*)p->h_steps.data(), p->n_steps, p->geom.maxA,
                                           p->h_sph.empty() ? nullptr : p->h_sph.data(), p->n_sph, ikc ? &p->ikd : nullptr,
                                           p->h_ikc_steps.data(), p->h_ikc_sph.data(), kernels, &k);
    if (rc != KIN_OK) return rc;
    jit_destroy(p->jit);
    p->jit = k;
    p->jit_mask = kernels;
    return KIN_OK;
}
}  // namespace

int kin_plan_specialize(kin_plan* p, uint32_t kernels) {
    if (!p) return set_error(KIN_E_INVALID, "kin_plan_specialize: null plan");
    if (const int rc = check_device(p->device, "kin_plan_specialize", "the plan")) return rc;
    uint32_t applies = 0;
    if (p->is_coll_ik) {
        applies = KIN_SPEC_IK | KIN_SPEC_IK_COLL | KIN_SPEC_IK_COLL_SCENE;
    } else if (p->is_coll) {
        applies = KIN_SPEC_COLL;
    } else {
        applies = KIN_SPEC_FK;
        if (p->ik_ok) applies |= KIN_SPEC_IK;
        if (p->ik_ok && !p->with_base) applies |= KIN_SPEC_NAKAMURA;
    }
    if (kernels == 0) kernels = applies;
    if (kernels & ~applies) return set_error(KIN_E_UNSUPPORTED, "kin_plan_specialize: kernel kind does not apply");
    if (p->parts.empty()) return specialize_one(p, kernels);
    for (auto& part : p->parts) {  // multi-chain collision plans: every chain program
        const int rc = specialize_one(part.get(), kernels);
        if (rc != KIN_OK) return rc;
    }
    p->jit_mask = kernels;
    return KIN_OK;
}

int kin_jit_selfcheck(void) { return jit_selfcheck(); }

int kin_plan_specialize_scene(kin_plan* p, const kin_sdf* sdf) {
    auto bad = [](int code, const std::string& w) { return set_error(code, "kin_plan_specialize_scene: " + w); };
    if (!p || !sdf) return bad(KIN_E_INVALID, "null plan / sdf");
    if (!p->is_coll || p->is_coll_ik) return bad(KIN_E_UNSUPPORTED, "plan was not made by kin_coll_plan_create");
    if (!sdf->attached) return bad(KIN_E_INVALID, "the kin_sdf is not attached to a scene");
    if (const int rc = check_device(p->device, "kin_plan_specialize_scene", "the plan")) return rc;
    if (const int rc = check_device(sdf->device, "kin_plan_specialize_scene", "the kin_sdf")) return rc;
    auto one = [&](kin_plan* s) -> int {
        {
            std::lock_guard<std::mutex> lk(s->scene_mu);
            if (s->scene_jit.count(sdf->uid)) return KIN_OK;
        }
        JitKernels* k = nullptr;
        int rc;
        if (s->dtype == KIN_F32) {
            const JitScene js{sdf->h_groups.data(), (int)sdf->h_groups.size(), sdf->h_ssf.data(), (int)sdf->h_ssf.size(),
                              sdf->h_bf.data(), (int)sdf->h_bf.size(), sdf->h_af.data(), (int)sdf->h_af.size(),
                              sdf->scene_base_col};
            rc = jit_build_scene<float>(s->pf, (const KStep<float>*)s->h_steps.data(), s->n_steps, s->geom.maxA,
                                        s->h_sph.empty() ? nullptr : s->h_sph.data(), s->n_sph, js, &k);
        } else {
            const JitScene js{sdf->h_groups.data(), (int)sdf->h_groups.size(), sdf->h_ssd.data(), (int)sdf->h_ssd.size(),
                              sdf->h_bd.data(), (int)sdf->h_bd.size(), sdf->h_ad.data(), (int)sdf->h_ad.size(),
                              sdf->scene_base_col};
            rc = jit_build_scene<double>(s->pd, (const KStep<double>*)s->h_steps.data(), s->n_steps, s->geom.maxA,
                                         s->h_sph.empty() ? nullptr : s->h_sph.data(), s->n_sph, js, &k);
        }
        if (rc != KIN_OK) return rc;
        std::lock_guard<std::mutex> lk(s->scene_mu);
        if (!s->scene_jit.emplace(sdf->uid, k).second) jit_destroy(k);
        return KIN_OK;
    };
    if (p->parts.empty()) return one(p);
    for (auto& part : p->parts)
        if (const int rc = one(part.get())) return rc;
    return KIN_OK;
}

int kin_plan_specialized(const kin_plan* p, uint32_t* kernels) {
    if (!p || !kernels) return set_error(KIN_E_INVALID, "kin_plan_specialized: null argument");
    *kernels = p->jit_mask;
    return KIN_OK;
}

int kin_get_transform_batch(kin_model* m, int32_t dtype, int32_t n_q, const int32_t* qids, const void* q,
                            int64_t ldq, int64_t n, int32_t n_out, const int32_t* out_ids, void* poses, int64_t ldp,
                            void* stream) {
    if (!m) return set_error(KIN_E_INVALID, "null model");
    kin_plan_desc d{dtype, n_q, qids, n_out, out_ids, 0, 0, nullptr, 0};
    kin_plan* p;
    const int rc = cached_plan(m, d, &p);
    if (rc != KIN_OK) return rc;
    if (n_out > 0 && !poses) return set_error(KIN_E_INVALID, "null poses");
    return kin_plan_run(p, q, ldq, n, poses, ldp, nullptr, 0, stream);
}

int kin_get_jacobian_batch(kin_model* m, int32_t dtype, int32_t link_id, int32_t n_joints, const int32_t* jids,
                           uint32_t flags, const void* q, int64_t ldq, int64_t n, void* pose, int64_t ldp, void* jac,
                           int64_t ldj, void* stream) {
    if (!m) return set_error(KIN_E_INVALID, "null model");
    if (link_id == 0) return set_error(KIN_E_KEY, "link id 0");
    const int32_t out_ids[1] = {link_id};
    kin_plan_desc d{dtype, n_joints, jids, pose ? 1 : 0, out_ids, link_id, n_joints, jids, flags};
    kin_plan* p;
    const int rc = cached_plan(m, d, &p);
    if (rc != KIN_OK) return rc;
    return kin_plan_run(p, q, ldq, n, pose, ldp, jac, ldj, stream);
}

int kin_sdf_create_boxes(int32_t n_boxes, const double* poses16, const double* widths3, kin_sdf** out) {
    if (!out || n_boxes < 1 || !poses16 || !widths3)
        return set_error(KIN_E_INVALID, "kin_sdf_create_boxes: need >= 1 box and non-null arrays");
    for (int32_t k = 0; k < 3 * n_boxes; ++k)
        if (!(widths3[k] >= 0)) return set_error(KIN_E_INVALID, "kin_sdf_create_boxes: negative / NaN width");
    auto sd = std::make_unique<kin_sdf>();
    sd->n_boxes = n_boxes;
    // axis-aligned boxes first (their own order), then the rotated ones
    std::vector<int32_t> order;
    std::vector<std::array<int, 3>> perms(n_boxes);
    for (int32_t k = 0; k < n_boxes; ++k)
        if (axis_permutation(poses16 + 16 * k, perms[k].data())) order.push_back(k);
    sd->n_aabb = (int32_t)order.size();
    for (int32_t k = 0; k < n_boxes; ++k)
        if (!axis_permutation(poses16 + 16 * k, perms[k].data())) order.push_back(k);
    std::vector<KBox<float>> bf(n_boxes);
    std::vector<KBox<double>> bd(n_boxes);
    std::vector<KAabb<float>> af(sd->n_aabb);
    std::vector<KAabb<double>> ad(sd->n_aabb);
    for (int32_t o = 0; o < n_boxes; ++o) {
        const int32_t k = order[o];
        const double* P = poses16 + 16 * k;
        const M34 inv = m_rigid_inverse(m_from_col16(P));  // BoxSDF.inv_pose (src/sdf.jl:60)
        to_row12<float>(inv, bf[o].inv);
        to_row12<double>(inv, bd[o].inv);
        for (int i = 0; i < 3; ++i) {
            bf[o].half[i] = (float)(0.5 * widths3[3 * k + i]);
            bd[o].half[i] = 0.5 * widths3[3 * k + i];
        }
        bf[o].pad = 0;
        bd[o].pad = 0;
        if (o < sd->n_aabb) {
            for (int i = 0; i < 3; ++i) {
                const int j = perms[k][i];  // box axis i lies along world axis j
                ad[o].c[i] = P[12 + i];
                af[o].c[i] = (float)P[12 + i];
                ad[o].half[j] = 0.5 * widths3[3 * k + i];
                af[o].half[j] = (float)(0.5 * widths3[3 * k + i]);
            }
            ad[o].pad[0] = ad[o].pad[1] = 0;
            af[o].pad[0] = af[o].pad[1] = 0;
        }
    }
    {  // enclosing world-aligned box of all box corners
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        std::vector<std::array<double, 3>> corners;
        for (int32_t k = 0; k < n_boxes; ++k) {
            const double* P = poses16 + 16 * k;  // column-major 4x4
            for (int c = 0; c < 8; ++c) {
                const double l[3] = {(c & 1 ? 0.5 : -0.5) * widths3[3 * k], (c & 2 ? 0.5 : -0.5) * widths3[3 * k + 1],
                                     (c & 4 ? 0.5 : -0.5) * widths3[3 * k + 2]};
                std::array<double, 3> w;
                for (int i = 0; i < 3; ++i) {
                    w[i] = P[12 + i] + P[i] * l[0] + P[4 + i] * l[1] + P[8 + i] * l[2];
                    lo[i] = std::min(lo[i], w[i]);
                    hi[i] = std::max(hi[i], w[i]);
                }
                corners.push_back(w);
            }
        }
        for (int i = 0; i < 3; ++i) {
            sd->bc[i] = 0.5 * (lo[i] + hi[i]);
            sd->bh[i] = 0.5 * (hi[i] - lo[i]) * (1.0 + 1e-12) + 1e-12;
        }
    }
    hipError_t e = hipGetDevice(&sd->device);
    if (e == hipSuccess) e = upload_boxes(&sd->d_f32, bf, af);
    if (e == hipSuccess) e = upload_boxes(&sd->d_f64, bd, ad);
    if (e != hipSuccess) return set_error(KIN_E_DEVICE, std::string("kin_sdf_create_boxes: ") + hipGetErrorString(e));
    *out = sd.release();
    return KIN_OK;
}

int kin_sdf_destroy(kin_sdf* s) {
    delete s;
    return KIN_OK;
}

int kin_sdf_create_attached(const kin_model* scene, int32_t n_q, const int32_t* q_joint_ids, int32_t n_boxes,
                            const int32_t* link_ids, const double* origins16, const double* widths3, kin_sdf** out) {
    auto bad = [](int code, const std::string& w) { return set_error(code, "kin_sdf_create_attached: " + w); };
    if (!scene || !out || n_boxes < 1 || !link_ids || !origins16 || !widths3 || n_q < 0 || (n_q && !q_joint_ids))
        return bad(KIN_E_INVALID, "null argument / no boxes");
    const kin_model& m = *scene;
    const int32_t J = m.n_joints(), L = m.n_links;
    std::vector<int32_t> qcol(J, -1);
    for (int32_t c = 0; c < n_q; ++c) {
        const int32_t j = q_joint_ids[c] - 1;
        if (j < 0 || j >= J) return bad(KIN_E_KEY, "scene joint id out of range");
        if (m.jtype[j] != KIN_JOINT_FIXED) qcol[j] = c;
    }
    for (int32_t k = 0; k < 3 * n_boxes; ++k)
        if (!(widths3[k] >= 0)) return bad(KIN_E_INVALID, "negative / NaN width");
    // per box: the group (last batch joint on its root path, -1: the root / base frame) and its pose in
    // the group frame (static joints at the scene's angles folded in, fp64, as joint_transform does)
    struct BoxS { int32_t group; M34 pose; int32_t src; };
    std::vector<BoxS> bs(n_boxes);
    std::vector<int32_t> group_key;  // joint (0-based) or -1
    for (int32_t k = 0; k < n_boxes; ++k) {
        const int32_t l = link_ids[k] - 1;
        if (l < 0 || l >= L) return bad(KIN_E_KEY, "box link id out of range");
        std::vector<int32_t> path;  // joints root .. l
        for (int32_t x = l; x >= 0 && m.link_pjoint[x] >= 0; x = m.plink(x)) path.push_back(m.link_pjoint[x]);
        std::reverse(path.begin(), path.end());
        int32_t last = -1;
        for (size_t p = 0; p < path.size(); ++p)
            if (qcol[path[p]] >= 0) last = (int32_t)p;
        M34 S = m_identity();
        for (size_t p = last + 1; p < path.size(); ++p) S = m_mul(S, m.joint_tf(path[p], m.angles[path[p]]));
        const int32_t key = last >= 0 ? path[last] : -1;
        auto it = std::find(group_key.begin(), group_key.end(), key);
        if (it == group_key.end()) {
            group_key.push_back(key);
            it = group_key.end() - 1;
        }
        bs[k] = BoxS{(int32_t)(it - group_key.begin()), m_mul(S, m_from_col16(origins16 + 16 * k)), k};
    }
    if ((int)group_key.size() > kMaxSceneGroups)
        return bad(KIN_E_UNSUPPORTED, "boxes ride on " + std::to_string(group_key.size()) + " moving frames (max " +
                                          std::to_string(kMaxSceneGroups) + ")");
    // group chains: static products up to each batch joint, then its motion (joint_transform)
    std::vector<KSceneGroup> groups(group_key.size());
    struct StepS { M34 F; double axis[3]; int32_t kind, qcol; };
    std::vector<StepS> steps;
    for (size_t g = 0; g < group_key.size(); ++g) {
        groups[g].step0 = (int32_t)steps.size();
        const int32_t key = group_key[g];
        if (key >= 0) {
            std::vector<int32_t> path;
            for (int32_t x = m.jclink[key] - 1; x >= 0 && m.link_pjoint[x] >= 0; x = m.plink(x)) path.push_back(m.link_pjoint[x]);
            std::reverse(path.begin(), path.end());
            M34 S = m_identity();
            for (int32_t j : path) {
                if (qcol[j] >= 0) {
                    StepS st;
                    st.F = m_mul(S, m.pose(j));
                    const double* ax = &m.jaxis[3 * j];
                    const double nn = sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
                    for (int i = 0; i < 3; ++i) st.axis[i] = nn > 0 ? ax[i] / nn : 0.0;
                    st.kind = m.jtype[j] == KIN_JOINT_PRISMATIC ? MOT_PRISM : MOT_REV;
                    st.qcol = qcol[j];
                    if (st.kind == MOT_PRISM) for (int i = 0; i < 3; ++i) st.axis[i] = ax[i];  // axis * q, unnormalised
                    steps.push_back(st);
                    S = m_identity();
                } else {
                    S = m_mul(S, m.joint_tf(j, m.angles[j]));
                }
            }
        }
        groups[g].step1 = (int32_t)steps.size();
    }
    // boxes sorted by group, axis-aligned ones first within a group
    std::vector<int32_t> order;
    std::vector<std::array<int, 3>> perms(n_boxes);
    std::vector<char> aa(n_boxes, 0);
    for (int32_t k = 0; k < n_boxes; ++k) {
        double P16[16] = {0};
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) P16[i + 4 * j] = bs[k].pose.r[3 * i + j];
            P16[12 + i] = bs[k].pose.t[i];
        }
        P16[15] = 1;
        aa[k] = axis_permutation(P16, perms[k].data());
    }
    std::vector<KBox<float>> bf;
    std::vector<KBox<double>> bd;
    std::vector<KAabb<float>> af;
    std::vector<KAabb<double>> ad;
    for (size_t g = 0; g < groups.size(); ++g) {
        groups[g].box0 = (int32_t)bf.size();
        groups[g].aabb0 = (int32_t)af.size();
        std::vector<int32_t> mem;
        for (int32_t k = 0; k < n_boxes; ++k)
            if (bs[k].group == (int32_t)g && aa[k]) mem.push_back(k);
        groups[g].na = (int32_t)mem.size();
        for (int32_t k = 0; k < n_boxes; ++k)
            if (bs[k].group == (int32_t)g && !aa[k]) mem.push_back(k);
        groups[g].nb = (int32_t)mem.size();
        {  // the group frame's box enclosing its boxes (|R| h around t), rounded outward to float
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int32_t k : mem)
                for (int i = 0; i < 3; ++i) {
                    double e = 0;
                    for (int j = 0; j < 3; ++j) e += fabs(bs[k].pose.r[3 * i + j]) * 0.5 * widths3[3 * k + j];
                    lo[i] = std::min(lo[i], bs[k].pose.t[i] - e);
                    hi[i] = std::max(hi[i], bs[k].pose.t[i] + e);
                }
            for (int i = 0; i < 3; ++i) {
                const double c = 0.5 * (lo[i] + hi[i]), h = 0.5 * (hi[i] - lo[i]);
                groups[g].bc[i] = (float)c;
                groups[g].bh[i] = (float)(h + 1e-6 * (fabs(c) + h) + 1e-6);
            }
        }
        for (size_t o = 0; o < mem.size(); ++o) {
            const int32_t k = mem[o];
            const M34 inv = m_rigid_inverse(bs[k].pose);
            KBox<float> xf{};
            KBox<double> xd{};
            to_row12<float>(inv, xf.inv);
            to_row12<double>(inv, xd.inv);
            for (int i = 0; i < 3; ++i) {
                xf.half[i] = (float)(0.5 * widths3[3 * k + i]);
                xd.half[i] = 0.5 * widths3[3 * k + i];
            }
            bf.push_back(xf);
            bd.push_back(xd);
            if ((int32_t)o < groups[g].na) {
                KAabb<float> yf{};
                KAabb<double> yd{};
                for (int i = 0; i < 3; ++i) {
                    const int j = perms[k][i];
                    yd.c[i] = bs[k].pose.t[i];
                    yf.c[i] = (float)bs[k].pose.t[i];
                    yd.half[j] = 0.5 * widths3[3 * k + i];
                    yf.half[j] = (float)(0.5 * widths3[3 * k + i]);
                }
                af.push_back(yf);
                ad.push_back(yd);
            }
        }
    }
    auto sd = std::make_unique<kin_sdf>();
    sd->attached = true;
    sd->n_boxes = n_boxes;
    sd->n_aabb = 0;
    sd->n_groups = (int32_t)groups.size();
    sd->scene_cols = n_q + (m.with_base ? 3 : 0);
    sd->scene_base_col = m.with_base ? n_q : -1;
    sd->scene_steps_off = ((sizeof(KSceneGroup) * groups.size() + 255) / 256) * 256;
    auto upload_scene = [&](auto tag, void** dst) -> hipError_t {
        using T = decltype(tag);
        std::vector<KSceneStep<T>> hs(std::max<size_t>(1, steps.size()));
        memset(hs.data(), 0, sizeof(KSceneStep<T>) * hs.size());
        for (size_t k = 0; k < steps.size(); ++k) {
            to_row12<T>(steps[k].F, hs[k].F);
            for (int i = 0; i < 3; ++i) hs[k].axis[i] = (T)steps[k].axis[i];
            hs[k].kind = steps[k].kind;
            hs[k].qcol = steps[k].qcol;
        }
        if constexpr (sizeof(T) == 4) sd->h_ssf.assign(hs.begin(), hs.begin() + steps.size());
        else sd->h_ssd.assign(hs.begin(), hs.begin() + steps.size());
        const size_t nb = sd->scene_steps_off + sizeof(KSceneStep<T>) * hs.size();
        hipError_t e = hipMalloc(dst, nb);
        if (e == hipSuccess) e = hipMemcpy(*dst, groups.data(), sizeof(KSceneGroup) * groups.size(), hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy((char*)*dst + sd->scene_steps_off, hs.data(), sizeof(KSceneStep<T>) * hs.size(),
                          hipMemcpyHostToDevice);
        return e;
    };
    sd->h_groups = groups;
    sd->h_bf = bf;
    sd->h_bd = bd;
    sd->h_af = af;
    sd->h_ad = ad;
    static std::atomic<uint64_t> sdf_uids{0};
    sd->uid = ++sdf_uids;
    hipError_t e = hipGetDevice(&sd->device);
    if (e == hipSuccess) e = upload_boxes(&sd->d_f32, bf, af);
    if (e == hipSuccess) e = upload_boxes(&sd->d_f64, bd, ad);
    if (e == hipSuccess) e = upload_scene(float(), &sd->d_scene_f32);
    if (e == hipSuccess) e = upload_scene(double(), &sd->d_scene_f64);
    if (e != hipSuccess) return bad(KIN_E_DEVICE, hipGetErrorString(e));
    *out = sd.release();
    return KIN_OK;
}

int kin_coll_plan_create(const kin_model* m, const kin_coll_desc* c, kin_plan** out) {
    if (!m || !c || !out) return set_error(KIN_E_INVALID, "kin_coll_plan_create: null argument");
    if (c->n_spheres < 1 || !c->sphere_link_ids || !c->radii)
        return set_error(KIN_E_INVALID, "kin_coll_plan_create: need >= 1 sphere with link ids and radii");
    if (c->n_q < 0 || (c->n_q && !c->q_joint_ids)) return set_error(KIN_E_INVALID, "kin_coll_plan_create: bad q");
    const int32_t L = m->n_links, J = m->n_joints();
    std::vector<char> moving(J, 0);
    for (int32_t k = 0; k < c->n_q; ++k) {
        const int32_t j = c->q_joint_ids[k] - 1;
        if (j < 0 || j >= J) return set_error(KIN_E_KEY, "kin_coll_plan_create: q joint id out of range");
        moving[j] = m->jtype[j] != KIN_JOINT_FIXED;
    }
    // Group the spheres by chain: the spine of a group is the remaining sphere anchor (nearest link
    // below a moving joint) with the most moving joints above it; the group takes every remaining
    // sphere whose anchor lies on the spine's root path.  One staged program per group.
    std::vector<int32_t> anchor(c->n_spheres), depth(c->n_spheres);
    for (int32_t k = 0; k < c->n_spheres; ++k) {
        int32_t x = c->sphere_link_ids[k] - 1;
        if (x < 0 || x >= L) return set_error(KIN_E_KEY, "kin_coll_plan_create: sphere link id out of range");
        while (x >= 0 && m->link_pjoint[x] >= 0 && !moving[m->link_pjoint[x]]) x = m->plink(x);
        int dd = 0;
        for (int32_t y = x; y >= 0 && m->link_pjoint[y] >= 0; y = m->plink(y)) dd += moving[m->link_pjoint[y]];
        anchor[k] = x;
        depth[k] = dd;
    }
    std::vector<char> done(c->n_spheres, 0);
    std::vector<std::unique_ptr<kin_plan>> parts;
    int32_t left = c->n_spheres;
    while (left > 0) {
        int32_t spine = -1, best = -1;
        for (int32_t k = 0; k < c->n_spheres; ++k)
            if (!done[k] && depth[k] > best) { best = depth[k]; spine = anchor[k]; }
        std::vector<char> on_path(L, 0);
        for (int32_t y = spine; y >= 0; y = m->plink(y)) on_path[y] = 1;
        std::vector<int32_t> ids, outs;
        std::vector<double> cen, rad;
        for (int32_t k = 0; k < c->n_spheres; ++k) {
            if (done[k] || !on_path[anchor[k]]) continue;
            done[k] = 1;
            --left;
            ids.push_back(c->sphere_link_ids[k]);
            outs.push_back(k);
            rad.push_back(c->radii[k]);
            for (int i = 0; i < 3; ++i) cen.push_back(c->centers ? c->centers[3 * k + i] : 0.0);
        }
        kin_coll_desc sub{c->dtype, c->n_q, c->q_joint_ids, (int32_t)ids.size(), ids.data(), cen.data(), rad.data()};
        kin_plan_desc d{c->dtype, c->n_q, c->q_joint_ids, 0, nullptr, spine + 1, c->n_q, c->q_joint_ids, 0};
        auto P = std::make_unique<kin_plan>();
        Stager st(*m, d);
        st.coll = &sub;
        st.sph_out = outs.data();
        const int rc = st.run(*P);
        if (rc != KIN_OK) return rc;
        parts.push_back(std::move(P));
    }
    std::unique_ptr<kin_plan> top;
    if (parts.size() == 1) {
        top = std::move(parts[0]);
    } else {
        top = std::make_unique<kin_plan>();
        top->dtype = parts[0]->dtype;
        top->nqcols = parts[0]->nqcols;
        top->with_base = parts[0]->with_base;
        top->n_q = parts[0]->n_q;
        top->is_coll = true;
        top->device = parts[0]->device;
        top->n_sph = c->n_spheres;
        top->parts = std::move(parts);
    }
    top->n_sph = c->n_spheres;
    *out = top.release();
    return KIN_OK;
}

namespace {
// The collision-aware IK program (kinhip_prog.h KIkcProg / KIkcStep): every moving joint above the target
// link or above a sphere link, depth first in joint order; static chains folded on the host in fp64 as
// joint_transform does (src/mechanism.jl:90-103), frames canonical (joint axis on local z, as the Stager).
struct IkcStepD {
    M34 F;
    double scale = 1;
    int32_t kind = MOT_NONE, flags = 0, var = -1, parent_step = -1, save = -1, sph0 = 0, sph1 = 0;
    uint32_t anc = 0;
};
struct IkcSphD {
    int32_t step;  // carrier step (-1: root frame)
    double c[3], r;
    int32_t out;
};

int stage_ikc_tree(const kin_model& m, const kin_coll_desc* c, int32_t link_id, kin_plan& P) {
    const int32_t L = m.n_links, J = m.n_joints();
    const int32_t tl = link_id - 1;
    if (tl < 0 || tl >= L) return set_error(KIN_E_KEY, "kin_coll_ik_plan_create: link id out of range");
    const int32_t nq = c->n_q, base_col = m.with_base ? nq : -1;
    const int32_t nv = nq + (m.with_base ? 3 : 0);
    if (nv > kIkcMaxVars)
        return set_error(KIN_E_UNSUPPORTED, "kin_coll_ik_plan_create: " + std::to_string(nv) + " variables (q columns + base; max " +
                                                std::to_string(kIkcMaxVars) + ")");
    if (c->n_spheres > kIkcMaxSpheres)
        return set_error(KIN_E_UNSUPPORTED, "kin_coll_ik_plan_create: more than " + std::to_string(kIkcMaxSpheres) + " spheres");
    std::vector<int32_t> qcol(J, -1);
    for (int32_t k = 0; k < nq; ++k) {
        const int32_t j = c->q_joint_ids[k] - 1;
        if (j < 0 || j >= J) return set_error(KIN_E_KEY, "kin_coll_ik_plan_create: q joint id out of range");
        qcol[j] = k;  // set_joint_angles: a repeated joint keeps the last column
    }
    std::vector<char> needed(L, 0);
    auto mark = [&](int32_t l) {
        for (int32_t x = l; x >= 0 && !needed[x]; x = m.plink(x)) needed[x] = 1;
    };
    mark(tl);
    std::vector<std::vector<int32_t>> sph_of(L);
    for (int32_t k = 0; k < c->n_spheres; ++k) {
        const int32_t lk = c->sphere_link_ids[k] - 1;
        if (lk < 0 || lk >= L) return set_error(KIN_E_KEY, "kin_coll_ik_plan_create: sphere link id out of range");
        mark(lk);
        sph_of[lk].push_back(k);
    }
    const uint32_t base_bits = m.with_base ? (7u << base_col) : 0u;
    std::vector<IkcStepD> steps;
    std::vector<IkcSphD> spheres;
    int32_t tgt_step = kIkcRoot;
    M34 Xt = m_identity();
    uint32_t prism = 0, joints = 0;
    // depth first from every root: `carrier` = step whose post-motion canonical frame carries link x,
    // S = that frame -> link x (static)
    std::function<int(int32_t, int32_t, const M34&, uint32_t)> visit = [&](int32_t x, int32_t carrier, const M34& S,
                                                                            uint32_t anc) -> int {
        if (x == tl) {
            tgt_step = carrier < 0 ? kIkcRoot : carrier;
            Xt = S;
        }
        for (int32_t k : sph_of[x]) {
            IkcSphD sd;
            const double c0 = c->centers ? c->centers[3 * k] : 0.0;
            const double c1 = c->centers ? c->centers[3 * k + 1] : 0.0;
            const double c2 = c->centers ? c->centers[3 * k + 2] : 0.0;
            for (int i = 0; i < 3; ++i) sd.c[i] = S.r[3 * i] * c0 + S.r[3 * i + 1] * c1 + S.r[3 * i + 2] * c2 + S.t[i];
            sd.r = c->radii[k];
            sd.out = k;
            sd.step = carrier;
            spheres.push_back(sd);
        }
        for (int32_t j : m.child_joints[x]) {
            const int32_t ch = m.jclink[j] - 1;
            if (!needed[ch]) continue;
            const bool moving = qcol[j] >= 0 && m.jtype[j] != KIN_JOINT_FIXED;
            if (!moving) {  // static: folded (joint held at m.angles)
                const int rc = visit(ch, carrier, m_mul(S, m.joint_tf(j, m.angles[j])), anc);
                if (rc != KIN_OK) return rc;
                continue;
            }
            if ((int32_t)steps.size() >= kIkcMaxSteps)
                return set_error(KIN_E_UNSUPPORTED, "kin_coll_ik_plan_create: more than " + std::to_string(kIkcMaxSteps) +
                                                        " moving joints on the needed tree");
            double scale;
            const M34 A = align_z(&m.jaxis[3 * j], &scale);
            IkcStepD st;
            st.F = m_mul(m_mul(S, m.pose(j)), A);
            st.scale = scale;
            st.kind = m.jtype[j] == KIN_JOINT_PRISMATIC ? MOT_PRISM : MOT_REV;
            if (st.kind == MOT_REV && scale != 1.0) st.flags |= SF_SCALE;
            st.var = qcol[j];
            st.parent_step = carrier;
            st.anc = anc | (1u << qcol[j]);
            joints |= 1u << qcol[j];
            if (st.kind == MOT_PRISM) prism |= 1u << qcol[j];
            const int32_t s = (int32_t)steps.size();
            steps.push_back(st);
            const int rc = visit(ch, s, m_rot_transpose(A), st.anc);
            if (rc != KIN_OK) return rc;
        }
        return KIN_OK;
    };
    for (int32_t l = 0; l < L; ++l)
        if (needed[l] && m.link_pjoint[l] < 0) {
            const int rc = visit(l, -1, m_identity(), base_bits);
            if (rc != KIN_OK) return rc;
        }
    // spheres in carrier order (root first, then the walk's step order), the caller's order inside a carrier
    std::stable_sort(spheres.begin(), spheres.end(), [](const IkcSphD& a, const IkcSphD& b) { return a.step < b.step; });
    int32_t sph_root0 = 0, sph_root1 = 0;
    for (size_t k = 0; k < spheres.size(); ++k) {
        const int32_t s = spheres[k].step;
        if (s < 0) {
            sph_root1 = (int32_t)k + 1;
        } else {
            if (steps[s].sph1 == 0) steps[s].sph0 = (int32_t)k;
            steps[s].sph1 = (int32_t)k + 1;
        }
    }
    // branch frames: a step whose frame a later, non-adjacent step starts from is saved into a slot, live
    // from the step to its last such child
    const int32_t ns = (int32_t)steps.size();
    std::vector<int32_t> last_use(ns, -1);
    for (int32_t s = 0; s < ns; ++s) {
        const int32_t p = steps[s].parent_step;
        if (p >= 0 && p != s - 1) last_use[p] = std::max(last_use[p], s);
    }
    std::vector<int32_t> slot_of(ns, -1), slot_free_at(kIkcMaxSlots, -1);
    for (int32_t s = 0; s < ns; ++s) {
        if (last_use[s] < 0) continue;
        int sl = -1;
        for (int k = 0; k < kIkcMaxSlots && sl < 0; ++k)
            if (slot_free_at[k] <= s) sl = k;
        if (sl < 0)
            return set_error(KIN_E_UNSUPPORTED, "kin_coll_ik_plan_create: the tree needs more than " +
                                                    std::to_string(kIkcMaxSlots) + " saved branch frames");
        slot_of[s] = sl;
        slot_free_at[sl] = last_use[s];
        steps[s].save = sl;
    }
    uint32_t tgt_mask = tgt_step == kIkcRoot ? base_bits : steps[tgt_step].anc;
    uint32_t free_mask = tgt_mask;
    for (const IkcSphD& sd : spheres) free_mask |= sd.step < 0 ? base_bits : steps[sd.step].anc;
    auto fill = [&](auto& K, auto* st_out, auto* sp_out) {
        using T = std::remove_reference_t<decltype(K.Xt[0])>;
        K = {};
        K.nS = ns;
        K.nv = nv;
        K.n_q = nq;
        K.base_col = base_col;
        K.n_sph = (int32_t)spheres.size();
        K.sph_root0 = sph_root0;
        K.sph_root1 = sph_root1;
        K.tgt_step = tgt_step;
        K.has_xt = !m_is_identity(Xt);
        K.tgt_mask = tgt_mask;
        K.free_mask = free_mask;
        K.joint_mask = joints;
        K.prism_mask = prism;
        to_row12<T>(Xt, K.Xt);
        for (int v = 0; v < kIkcMaxVars; ++v) {
            K.vlo[v] = (T)-INFINITY;
            K.vhi[v] = (T)INFINITY;
        }
        for (int32_t j = 0; j < J; ++j)
            if (qcol[j] >= 0 && ((joints >> qcol[j]) & 1u)) {
                K.vlo[qcol[j]] = (T)m.jlo[j];
                K.vhi[qcol[j]] = (T)m.jhi[j];
            }
        // the normal equations' structure: entry (v, c) gets terms from the pose rows when both move the
        // target, from a sphere's row when both move that sphere
        auto add_block = [&](uint32_t mask) {
            for (int v = 0; v < nv; ++v)
                if ((mask >> v) & 1u) K.nzrow[v] |= mask & ((2u << v) - 1u);
        };
        add_block(tgt_mask);
        for (const IkcSphD& sd : spheres) add_block(sd.step < 0 ? base_bits : steps[sd.step].anc);
        for (int32_t s = 0; s < ns; ++s) {
            const IkcStepD& a = steps[s];
            auto& b = st_out[s];
            memset(&b, 0, sizeof(b));
            to_row12<T>(a.F, b.F);
            b.scale = (T)a.scale;
            b.kind = a.kind;
            b.flags = a.flags;
            b.var = a.var;
            b.parent = a.parent_step < 0 ? kIkcRoot : a.parent_step == s - 1 ? kIkcPrev : slot_of[a.parent_step];
            b.save = a.save;
            b.sph0 = a.sph0;
            b.sph1 = a.sph1;
            b.anc = a.anc;
        }
        for (size_t k = 0; k < spheres.size(); ++k) {
            auto& b = sp_out[k];
            memset(&b, 0, sizeof(b));
            for (int i = 0; i < 3; ++i) b.c[i] = (T)spheres[k].c[i];
            b.r = (T)spheres[k].r;
            b.out = spheres[k].out;
            b.anc = spheres[k].step < 0 ? base_bits : steps[spheres[k].step].anc;
        }
    };
    const bool f32 = c->dtype == KIN_F32;
    const size_t est = f32 ? sizeof(KIkcStep<float>) : sizeof(KIkcStep<double>);
    const size_t esp = f32 ? sizeof(KSphere<float>) : sizeof(KSphere<double>);
    P.h_ikc_steps.assign(std::max<size_t>(1, ns) * est, 0);
    P.h_ikc_sph.assign(std::max<size_t>(1, spheres.size()) * esp, 0);
    if (f32)
        fill(P.ikf, (KIkcStep<float>*)P.h_ikc_steps.data(), (KSphere<float>*)P.h_ikc_sph.data());
    else
        fill(P.ikd, (KIkcStep<double>*)P.h_ikc_steps.data(), (KSphere<double>*)P.h_ikc_sph.data());
    return KIN_OK;
}

// the staged tree program to the device: [steps | spheres] in one allocation
int upload_ikc_tree(kin_plan& P) {
    P.ikc_sph_off = (P.h_ikc_steps.size() + 255) / 256 * 256;
    const size_t bytes = P.ikc_sph_off + P.h_ikc_sph.size();
    std::vector<unsigned char> host(bytes, 0);
    memcpy(host.data(), P.h_ikc_steps.data(), P.h_ikc_steps.size());
    memcpy(host.data() + P.ikc_sph_off, P.h_ikc_sph.data(), P.h_ikc_sph.size());
    hipError_t e = hipMalloc(&P.d_ikc, bytes);
    if (e != hipSuccess) {
        P.d_ikc = nullptr;
        return set_error(KIN_E_DEVICE, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    e = hipMemcpy(P.d_ikc, host.data(), bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) return set_error(KIN_E_DEVICE, std::string("hipMemcpy: ") + hipGetErrorString(e));
    return KIN_OK;
}
}  // namespace

int kin_coll_ik_plan_create(const kin_model* m, const kin_coll_desc* c, int32_t link_id, kin_plan** out) {
    if (!m || !c || !out) return set_error(KIN_E_INVALID, "kin_coll_ik_plan_create: null argument");
    if (c->n_spheres < 0 || (c->n_spheres && (!c->sphere_link_ids || !c->radii)))
        return set_error(KIN_E_INVALID, "kin_coll_ik_plan_create: spheres need link ids and radii");
    if (c->n_q < 1 || !c->q_joint_ids) return set_error(KIN_E_INVALID, "kin_coll_ik_plan_create: no q joints");
    const int32_t out_ids[1] = {link_id};
    // an IK plan of `link` over the q joints (stage 1: get_jacobian! over them, geometric rows) ...
    kin_plan_desc d{c->dtype, c->n_q, c->q_joint_ids, 1, out_ids, link_id, c->n_q, c->q_joint_ids, KIN_WITH_ROT};
    auto P = std::make_unique<kin_plan>();
    // ... and the tree of the target link and every sphere (stage 2, k_ik_tree; staged on the host first)
    int rc = stage_ikc_tree(*m, c, link_id, *P);
    if (rc != KIN_OK) return rc;
    Stager st(*m, d);
    rc = st.run(*P);
    if (rc != KIN_OK) return rc;
    if (!P->ik_ok) return set_error(KIN_E_INVALID, "kin_coll_ik_plan_create: " + P->ik_why);
    rc = upload_ikc_tree(*P);
    if (rc != KIN_OK) return rc;
    P->is_coll_ik = true;
    P->n_sph = c->n_spheres;
    *out = P.release();
    return KIN_OK;
}

namespace {
int ik_coll_batch(const kin_plan* p, const kin_sdf* sdf, const kin_ik_params* prm, const kin_ik_coll_params* cp,
                  const void* target, int64_t ldt, const void* scene_q, int64_t lds, bool scene, const void* q0,
                  const void* q_alt, void* q, int64_t ldq, int64_t n, int32_t* iters, void* err, int64_t lde, void* stream,
                  const char* fn) {
    auto bad = [&](int code, const std::string& w) { return set_error(code, std::string(fn) + ": " + w); };
    if (!p || !sdf || !prm || !cp) return bad(KIN_E_INVALID, "null argument");
    if (!p->is_coll_ik) return bad(KIN_E_INVALID, "plan was not made by kin_coll_ik_plan_create");
    if (sdf->attached && !scene) return bad(KIN_E_INVALID, "the kin_sdf is attached to a scene: use kin_ik_coll_batch_scene");
    if (!sdf->attached && scene) return bad(KIN_E_INVALID, "the kin_sdf is not attached to a scene (use kin_ik_coll_batch)");
    if (n < 0) return bad(KIN_E_INVALID, "n < 0");
    if (n == 0) return KIN_OK;
    if (!target || ldt < n || !q || ldq < n || (err && lde < n)) return bad(KIN_E_INVALID, "bad pointer / stride");
    if (scene && sdf->scene_cols > 0 && (!scene_q || (lds != 0 && lds < n))) return bad(KIN_E_INVALID, "bad scene_q / lds");
    if (const int rc = check_device(p->device, fn, "the plan")) return rc;
    if (const int rc = check_device(sdf->device, fn, "the kin_sdf")) return rc;
    if (prm->max_iters < 0 || !(prm->lambda > 0) || !(prm->max_step > 0) || prm->restarts < 0 ||
        prm->with_rot < 0 || prm->with_rot > 2 || prm->index_base < 0)
        return bad(KIN_E_INVALID, "bad IK parameters (lambda must be > 0)");
    if (prm->damp_err != 0.0) return bad(KIN_E_INVALID, "kin_ik_params.damp_err must be 0 for the collision-aware IK");
    if (!std::isfinite(cp->margin) || !(cp->band >= 0) || !(cp->weight > 0) || !(cp->feas >= 0))
        return bad(KIN_E_INVALID, "bad collision parameters");
    if (prm->lanes != 0 && prm->lanes != 1 && prm->lanes != 2 && prm->lanes != 4 && prm->lanes != 8 &&
        prm->lanes != 16 && prm->lanes != 64)
        return bad(KIN_E_INVALID, "kin_ik_params.lanes must be 0 (auto), 1, 2, 4, 8, 16 or 64");
    IkArgs a{prm->max_iters, prm->lambda, prm->tol_pos, prm->tol_rot, prm->max_step, prm->with_rot,
             prm->restarts, prm->seed, prm->lanes, prm->index_base, 0.0};
    a.q_alt = q_alt;
    const IkcArgs c{cp->margin, cp->band, cp->weight, cp->feas};
    const CollArgs ca{INFINITY, 0.0, sdf->n_boxes, sdf->n_aabb, 0, 0, {sdf->bc[0], sdf->bc[1], sdf->bc[2]},
                      {sdf->bh[0], sdf->bh[1], sdf->bh[2]}};
    const bool f32 = p->dtype == KIN_F32;
    const void* sc = f32 ? sdf->d_scene_f32 : sdf->d_scene_f64;
    const SceneLaunch sl{sc, sc ? (const char*)sc + sdf->scene_steps_off : nullptr, scene_q, lds, sdf->n_groups,
                         sdf->scene_base_col, lds == 0 ? 1 : 0};
    const JitFns* jf = jit_fns(p->jit);  // (the specialised kernels take the static union only)
    const void* st = p->d_ikc;
    const void* sp = (const char*)p->d_ikc + p->ikc_sph_off;
    hipError_t e;
    if (f32)
        e = launch_ik_tree<float>(p->ikf, (const KIkcStep<float>*)st, (const KSphere<float>*)sp, (const KBox<float>*)sdf->d_f32,
                                  ca, scene ? &sl : nullptr, c, a, (const float*)target, ldt,
                                  (const float*)(q0 == q ? nullptr : q0), (float*)q, ldq, n, iters, (float*)err, lde, jf,
                                  (hipStream_t)stream);
    else
        e = launch_ik_tree<double>(p->ikd, (const KIkcStep<double>*)st, (const KSphere<double>*)sp,
                                   (const KBox<double>*)sdf->d_f64, ca, scene ? &sl : nullptr, c, a, (const double*)target,
                                   ldt, (const double*)(q0 == q ? nullptr : q0), (double*)q, ldq, n, iters, (double*)err,
                                   lde, jf, (hipStream_t)stream);
    if (e != hipSuccess) return set_error(KIN_E_DEVICE, std::string("k_ik_tree launch: ") + hipGetErrorString(e));
    return KIN_OK;
}
}  // namespace

int kin_ik_coll_batch(const kin_plan* p, const kin_sdf* sdf, const kin_ik_params* prm, const kin_ik_coll_params* cp,
                      const void* target, int64_t ldt, const void* q0, void* q, int64_t ldq, int64_t n, int32_t* iters,
                      void* err, int64_t lde, void* stream) {
    return ik_coll_batch(p, sdf, prm, cp, target, ldt, nullptr, 0, false, q0, nullptr, q, ldq, n, iters, err, lde,
                         stream, "kin_ik_coll_batch");
}

int kin_ik_coll_batch_scene(const kin_plan* p, const kin_sdf* sdf, const kin_ik_params* prm,
                            const kin_ik_coll_params* cp, const void* target, int64_t ldt, const void* scene_q,
                            int64_t lds, const void* q0, void* q, int64_t ldq, int64_t n, int32_t* iters, void* err,
                            int64_t lde, void* stream) {
    return ik_coll_batch(p, sdf, prm, cp, target, ldt, scene_q, lds, true, q0, nullptr, q, ldq, n, iters, err, lde,
                         stream, "kin_ik_coll_batch_scene");
}

int kin_ik_coll_batch_alt(const kin_plan* p, const kin_sdf* sdf, const kin_ik_params* prm,
                          const kin_ik_coll_params* cp, const void* target, int64_t ldt, const void* scene_q,
                          int64_t lds, const void* q0, const void* q_alt, void* q, int64_t ldq, int64_t n,
                          int32_t* iters, void* err, int64_t lde, void* stream) {
    return ik_coll_batch(p, sdf, prm, cp, target, ldt, scene_q, lds, sdf && sdf->attached, q0, q_alt, q, ldq, n,
                         iters, err, lde, stream, "kin_ik_coll_batch_alt");
}

namespace {
// k_coll over every chain program of a collision plan; min_dist accumulates after the first
int coll_launch(const kin_plan* p, const kin_sdf* sdf, CollArgs a, const void* q, int64_t ldq, int64_t n, void* dists,
                int64_t ldd, void* grads, int64_t ldg, void* min_dist, const TileArgs& ta, void* stream) {
    const size_t np = p->parts.empty() ? 1 : p->parts.size();
    // the specialised kernels address rows through the scalar offset (KINHIP_COLL_SOFF): every row
    // offset plus the lane span must stay below 2^31 bytes, else the generic kernels run
    const int64_t esz = p->dtype == KIN_F32 ? 4 : 8;
    const bool tiled = ta.tile < n;
    const int64_t span = tiled ? ta.tile : std::min<int64_t>(n, kChunk);
    const auto fits = [&](int64_t rows, int64_t ld) { return ((rows + 1) * (tiled ? ta.tile : ld) + span) * esz < (int64_t(1) << 31); };
    const bool soff = fits(p->nqcols, ldq) && (!dists || fits(p->n_sph, ldd)) &&
                      (!grads || fits((int64_t)p->n_sph * p->nqcols, ldg));
    for (size_t k = 0; k < np; ++k) {
        const kin_plan* s = p->parts.empty() ? p : p->parts[k].get();
        a.accumulate = k > 0;
        const JitFns* jf = soff ? jit_fns(s->jit) : nullptr;
        hipError_t e;
        if (s->dtype == KIN_F32)
            e = launch_coll<float>(s->pf, (const KStep<float>*)s->d_steps, (const KSphere<float>*)s->d_sph,
                                   (const KBox<float>*)sdf->d_f32, s->geom, a, (const float*)q, ldq, n, (float*)dists,
                                   ldd, (float*)grads, ldg, (float*)min_dist, ta, jf, (hipStream_t)stream);
        else
            e = launch_coll<double>(s->pd, (const KStep<double>*)s->d_steps, (const KSphere<double>*)s->d_sph,
                                    (const KBox<double>*)sdf->d_f64, s->geom, a, (const double*)q, ldq, n,
                                    (double*)dists, ldd, (double*)grads, ldg, (double*)min_dist, ta, jf,
                                    (hipStream_t)stream);
        if (e != hipSuccess) return set_error(KIN_E_DEVICE, std::string("k_coll launch: ") + hipGetErrorString(e));
    }
    return KIN_OK;
}

CollArgs coll_args(const kin_sdf* sdf, double truncation, double offset) {
    return CollArgs{truncation, offset, sdf->n_boxes, sdf->n_aabb, 0, 0, {sdf->bc[0], sdf->bc[1], sdf->bc[2]},
                    {sdf->bh[0], sdf->bh[1], sdf->bh[2]}};
}

// shared checks of the collision entry points; ta.tile >= n is the plain layout
int coll_check(const kin_plan* p, const kin_sdf* sdf, const void* q, int64_t ldq, int64_t tsq, int64_t n,
               const void* out1, int64_t ld1, int64_t ts1, int rows1, const void* out2, int64_t ld2, int64_t ts2,
               int rows2, const TileArgs& ta, const char* fn) {
    auto bad = [&](const char* what) { return set_error(KIN_E_INVALID, std::string(fn) + ": " + what); };
    if (!p || !sdf) return bad("null plan / sdf");
    if (!p->is_coll) return bad("plan was not made by kin_coll_plan_create");
    if (sdf->attached) return bad("the kin_sdf is attached to a scene: use kin_coll_batch_scene");
    if (n < 0) return bad("n < 0");
    if (n == 0) return KIN_OK;
    if (const int rc = check_device(p->device, fn, "the plan")) return rc;
    if (const int rc = check_device(sdf->device, fn, "the kin_sdf")) return rc;
    const int64_t span = std::min(ta.tile, n);
    if ((p->nqcols > 0 && (!q || ldq < span)) || (out1 && ld1 < span) || (out2 && ld2 < span))
        return bad("bad pointer / stride");
    if (ta.tile < n) {
        if (ta.tile < 256 || ta.tile % 256 || ta.tile > (int64_t(1) << 26)) return bad("tile must be a multiple of 256 <= 2^26");
        if ((p->nqcols > 0 && tsq < p->nqcols * ldq) || (out1 && ts1 < rows1 * ld1) || (out2 && ts2 < rows2 * ld2))
            return bad("tile strides overlap");
    }
    return KIN_OK;
}
}  // namespace

int kin_coll_batch(const kin_plan* p, const kin_sdf* sdf, double truncation, const void* q, int64_t ldq, int64_t n,
                   void* dists, int64_t ldd, void* grads, int64_t ldg, void* min_dist, void* stream) {
    const TileArgs ta = plain_soa(n);
    const int rc = coll_check(p, sdf, q, ldq, 0, n, dists, ldd, 0, 0, grads, ldg, 0, 0, ta, "kin_coll_batch");
    if (rc != KIN_OK || n == 0) return rc;
    return coll_launch(p, sdf, coll_args(sdf, truncation, 0.0), q, ldq, n, dists, ldd, grads, ldg, min_dist, ta,
                       stream);
}

int kin_coll_batch_scene(const kin_plan* p, const kin_sdf* sdf, double truncation, const void* q, int64_t ldq,
                         const void* scene_q, int64_t lds, int64_t n, void* dists, int64_t ldd, void* grads, int64_t ldg,
                         void* min_dist, void* stream) {
    auto bad = [](const std::string& w) { return set_error(KIN_E_INVALID, "kin_coll_batch_scene: " + w); };
    if (!p || !sdf) return bad("null plan / sdf");
    if (!p->is_coll) return bad("plan was not made by kin_coll_plan_create");
    if (!sdf->attached) return bad("the kin_sdf is not attached to a scene (use kin_coll_batch)");
    if (n < 0) return bad("n < 0");
    if (n == 0) return KIN_OK;
    if (sdf->scene_cols > 0 && (!scene_q || (lds != 0 && lds < n))) return bad("bad scene_q / lds");
    if ((p->nqcols > 0 && (!q || ldq < n)) || (dists && ldd < n) || (grads && ldg < n)) return bad("bad pointer / stride");
    if (const int rc = check_device(p->device, "kin_coll_batch_scene", "the plan")) return rc;
    if (const int rc = check_device(sdf->device, "kin_coll_batch_scene", "the kin_sdf")) return rc;
    CollArgs a = coll_args(sdf, truncation, 0.0);
    const size_t np = p->parts.empty() ? 1 : p->parts.size();
    // the specialised kernels' soffset row addressing (as coll_launch): every row offset plus the lane
    // span below 2^31 bytes, else the generic kernels
    const int64_t esz = p->dtype == KIN_F32 ? 4 : 8, span = std::min<int64_t>(n, kChunk);
    const auto fits = [&](int64_t rows, int64_t ld) { return ((rows + 1) * ld + span) * esz < (int64_t(1) << 31); };
    const bool soff = fits(p->nqcols, ldq) && (!dists || fits(p->n_sph, ldd)) &&
                      (!grads || fits((int64_t)p->n_sph * p->nqcols, ldg));
    for (size_t k = 0; k < np; ++k) {
        const kin_plan* s = p->parts.empty() ? p : p->parts[k].get();
        a.accumulate = k > 0;
        const JitFns* jf = soff ? jit_fns(s->jit) : nullptr;
        const JitFns* jfs = soff ? s->scene_fns(sdf->uid) : nullptr;  // (kin_plan_specialize_scene)
        const void* sc = s->dtype == KIN_F32 ? sdf->d_scene_f32 : sdf->d_scene_f64;
        const SceneLaunch sl{sc, (const char*)sc + sdf->scene_steps_off, scene_q, lds, sdf->n_groups,
                             sdf->scene_base_col, lds == 0 ? 1 : 0};
        hipError_t e;
        if (s->dtype == KIN_F32)
            e = launch_coll_scene<float>(s->pf, (const KStep<float>*)s->d_steps, (const KSphere<float>*)s->d_sph,
                                         (const KBox<float>*)sdf->d_f32, s->geom, a, sl, (const float*)q, ldq, n,
                                         (float*)dists, ldd, (float*)grads, ldg, (float*)min_dist, jf, jfs,
                                         (hipStream_t)stream);
        else
            e = launch_coll_scene<double>(s->pd, (const KStep<double>*)s->d_steps, (const KSphere<double>*)s->d_sph,
                                          (const KBox<double>*)sdf->d_f64, s->geom, a, sl, (const double*)q, ldq, n,
                                          (double*)dists, ldd, (double*)grads, ldg, (double*)min_dist, jf, jfs,
                                          (hipStream_t)stream);
        if (e != hipSuccess) return set_error(KIN_E_DEVICE, std::string("k_coll_scene launch: ") + hipGetErrorString(e));
    }
    return KIN_OK;
}

int kin_ineq_const_batch(const kin_plan* p, const kin_sdf* sdf, double margin, const void* q, int64_t ldq, int64_t n,
                         void* vals, int64_t ldv, void* jac, int64_t ldj, void* stream) {
    if (!std::isfinite(margin)) return set_error(KIN_E_INVALID, "kin_ineq_const_batch: margin must be finite");
    if (!vals) return set_error(KIN_E_INVALID, "kin_ineq_const_batch: null vals");
    const TileArgs ta = plain_soa(n > 0 ? n : 1);
    const int ndof = p ? p->nqcols : 0;
    const int rc = coll_check(p, sdf, q, ldq, 0, n, vals, ldv, 0, p ? p->n_sph : 0, jac, ldj, 0,
                              p ? p->n_sph * ndof : 0, ta, "kin_ineq_const_batch");
    if (rc != KIN_OK || n == 0) return rc;
    // src/planning.jl:56, :66: truncation_dist = margin + 0.05; val = dist - margin
    return coll_launch(p, sdf, coll_args(sdf, margin + 0.05, margin), q, ldq, n, vals, ldv, jac, ldj, nullptr, ta,
                       stream);
}

int kin_pose_const_batch(const kin_plan* p, const void* target, int64_t ldt, const void* q, int64_t ldq, int64_t n,
                         void* poses, int64_t ldp, void* vals, int64_t ldv, void* jac, int64_t ldj, void* stream) {
    if (!p) return set_error(KIN_E_INVALID, "kin_pose_const_batch: null plan");
    if (p->is_coll || p->n_out != 1 || !p->has_jac || p->out_link0 != p->jac_link)
        return set_error(KIN_E_INVALID, "kin_pose_const_batch: plan needs n_out = 1 and a Jacobian of that same link");
    if (p->rows == 6 && !p->has_rpy)
        return set_error(KIN_E_INVALID, "kin_pose_const_batch: with_rot plans need KIN_RPY_JAC (rpy_jac=true)");
    if (n < 0) return set_error(KIN_E_INVALID, "n < 0");
    if (n == 0) return KIN_OK;
    if (!target || ldt < n || !vals || ldv < n) return set_error(KIN_E_INVALID, "kin_pose_const_batch: bad target / vals");
    int rc = kin_plan_run(p, q, ldq, n, poses, ldp, jac, ldj, stream);
    if (rc != KIN_OK) return rc;
    hipError_t e;
    if (p->dtype == KIN_F32)
        e = launch_pose_residual<float>((const float*)poses, ldp, (const float*)target, ldt, n, p->rows, (float*)vals,
                                        ldv, (hipStream_t)stream);
    else
        e = launch_pose_residual<double>((const double*)poses, ldp, (const double*)target, ldt, n, p->rows,
                                         (double*)vals, ldv, (hipStream_t)stream);
    if (e != hipSuccess) return set_error(KIN_E_DEVICE, std::string("k_pose_residual launch: ") + hipGetErrorString(e));
    return KIN_OK;
}

// The state of scratch set k's last call: hipSuccess once it has completed, hipErrorNotReady while it runs, with
// `wait` a host wait for it first.  An event last recorded on hipStreamPerThread by a thread that has since exited
// can report an error instead (hipErrorCapturedEvent: this runtime consults the recording stream, destroyed with
// its thread -- seen once in a full GPU suite, profiles/r06_gpu_tests_capturedevent.log).  That thread's exit
// drained its per-thread stream (tools/pts_probe.hip), so the call has completed: the error is cleared, the set
// gets a fresh event, and the result is hipSuccess.  Any other error is returned.  (Caller: the set is its own --
// ik_mu held, or ik_busy.)
static hipError_t ik_set_state(const kin_plan* p, int k, bool wait) {
    hipError_t e = hipEventQuery(p->ik_ev[k]);
    if (e == hipErrorNotReady && wait) e = hipEventSynchronize(p->ik_ev[k]);
    if (e != hipSuccess && e != hipErrorNotReady && p->ik_stream[k] == (void*)hipStreamPerThread) {
        (void)hipGetLastError();
        hipEvent_t fresh = nullptr;
        if (hipEventCreateWithFlags(&fresh, hipEventDisableTiming) == hipSuccess) {
            (void)hipEventDestroy(p->ik_ev[k]);
            (void)hipGetLastError();
            p->ik_ev[k] = fresh;
        }
        e = hipSuccess;
    }
    return e;
}

static int ik_dls_batch(const kin_plan* p, const kin_ik_params* prm, const void* target, int64_t ldt, const void* q0,
                        void* q, int64_t ldq, int64_t n, int32_t* iters, void* err, int64_t lde, void* stream,
                        void* trace = nullptr, int64_t ldtr = 0) {
    if (!p || !prm) return set_error(KIN_E_INVALID, "kin_ik_dls_batch: null argument");
    if (!p->ik_ok) return set_error(KIN_E_INVALID, "kin_ik_dls_batch: plan not usable for IK: " + p->ik_why);
    if (n < 0) return set_error(KIN_E_INVALID, "n < 0");
    if (n == 0) return KIN_OK;
    if (!target || ldt < n || !q || ldq < n || (err && lde < n)) return set_error(KIN_E_INVALID, "bad pointer / stride");
    if (const int rc = check_device(p->device, "kin_ik_dls_batch", "the plan")) return rc;
    if (prm->max_iters < 0 || !(prm->lambda >= 0) || !(prm->max_step > 0) || prm->restarts < 0)
        return set_error(KIN_E_INVALID, "bad IK parameters");
    if (prm->with_rot < 0 || prm->with_rot > 2)
        return set_error(KIN_E_INVALID, "kin_ik_params.with_rot must be 0, 1 or 2 (reference rpy objective)");
    if (prm->lanes != 0 && prm->lanes != 1 && prm->lanes != 2 && prm->lanes != 4 && prm->lanes != 8)
        return set_error(KIN_E_INVALID, "kin_ik_params.lanes must be 0 (auto), 1, 2, 4 or 8");
    if (prm->index_base < 0) return set_error(KIN_E_INVALID, "kin_ik_params.index_base < 0");
    if (!(prm->damp_err >= 0) || !std::isfinite(prm->damp_err))
        return set_error(KIN_E_INVALID, "kin_ik_params.damp_err must be finite and >= 0");
    IkArgs a{prm->max_iters, prm->lambda, prm->tol_pos, prm->tol_rot, prm->max_step, prm->with_rot,
             prm->restarts, prm->seed, prm->lanes, prm->index_base, prm->damp_err};
    if (trace) {  // kin_ik_dls_batch_trace: one lane per target, attempts in sequence (rows by iteration)
        if (ldtr < n) return set_error(KIN_E_INVALID, "kin_ik_dls_batch_trace: ldtr < n");
        a.lanes = 1;
        a.trace = trace;
        a.trace_ld = ldtr;
    }
    // the specialised IK kernels address rows with 32-bit offsets (ldn_soa): every lane offset of a
    // launch chunk plus rows * ld must stay below 2^31 bytes, else the generic kernel runs
    const int64_t esz = p->dtype == KIN_F32 ? 4 : 8;
    const int64_t span = std::min<int64_t>(n, kIkChunk);
    const bool narrow = (12 * ldt + span) * esz < (int64_t(1) << 31) && (p->nqcols * ldq + span) * esz < (int64_t(1) << 31) &&
                        (2 * lde + span) * esz < (int64_t(1) << 31);
    const JitFns* jf = narrow ? jit_fns(p->jit) : nullptr;
    // two-phase schedule scratch (small batches with restarts; launch_ik_dls): only a call that runs
    // that schedule touches it, so every other call stays allocation-free (capture-safe)
    IkScratch scr;
    int eager_set = -1;  // eager scratch set taken by this call (released after the launch)
    if (ik_wants_two_phase(a, n, kin_plan::kIkScratchCap)) {
        // kIkSubRings rings of 2 * cap / kIkSubRings entries (a phase-1 launch spreads its hand-overs over
        // the rings by wave; twice the even share covers the uneven last waves), list + aux, and the
        // rings' control words (one 128-byte line each)
        const int64_t ring_cap = 2 * kin_plan::kIkScratchCap / kIkSubRings;
        const size_t ctl_bytes = sizeof(uint32_t) * kIkCtlStride * kIkSubRings;
        const size_t set_bytes = ctl_bytes + 2 * sizeof(int32_t) * (size_t)(ring_cap * kIkSubRings);
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing((hipStream_t)stream, &cs) != hipSuccess) cs = hipStreamCaptureStatusNone;
        const bool capturing = cs == hipStreamCaptureStatusActive;
        int set = -1;
        int wait_set = -1;  // the set's previous call ran on another stream: order this call after it
        {
            std::unique_lock<std::mutex> lk(p->ik_mu);
            if (!p->d_ikscr) {
                if (capturing)
                    return set_error(KIN_E_INVALID, "kin_ik_dls_batch: the plan's first two-phase call allocates its "
                                                    "scratch and cannot run inside a stream capture (make one call "
                                                    "outside the capture first, or pass lanes > 0)");
                hipError_t e0 = hipMalloc(&p->d_ikscr, set_bytes * kin_plan::kIkScratchSets);
                // the rings' control words start at zero and are never reset afterwards (launch_ik_dls)
                if (e0 == hipSuccess) e0 = hipMemset(p->d_ikscr, 0, set_bytes * kin_plan::kIkScratchSets);
                if (e0 != hipSuccess) {
                    if (p->d_ikscr) (void)hipFree(p->d_ikscr);
                    p->d_ikscr = nullptr;
                    return set_error(KIN_E_DEVICE, std::string("hipMalloc: ") + hipGetErrorString(e0));
                }
            }
            if (!capturing) {
                // One handle names one stream for every host thread except hipStreamPerThread, which is
                // each calling thread's own default stream: only a set last used through another handle
                // than that one can be matched by handle.  (The null stream is the device's legacy default
                // stream, shared by every thread: this library is not built for per-thread default streams.)
                const bool per_thread = (hipStream_t)stream == hipStreamPerThread;
                bool waited = false;
                for (;;) {
                    int lru = -1;
                    for (int k = 0; k < kin_plan::kIkEagerSets && set < 0; ++k)
                        if (!p->ik_busy[k] && !per_thread && p->ik_ev[k] && p->ik_stream[k] == stream) set = k;
                    for (int k = 0; k < kin_plan::kIkEagerSets && set < 0; ++k)
                        if (!p->ik_busy[k] && (!p->ik_ev[k] || ik_set_state(p, k, false) == hipSuccess)) set = k;
                    for (int k = 0; k < kin_plan::kIkEagerSets; ++k)
                        if (!p->ik_busy[k] && (lru < 0 || p->ik_tick[k] < p->ik_tick[lru])) lru = k;
                    if (set < 0) set = lru;
                    if (set >= 0) break;
                    // every set is between take and event record in other threads (a launch's host
                    // time): wait for one rather than share it
                    waited = true;
                    p->ik_cv.wait(lk);
                }
                if (waited) ++p->ik_stats.busy_waits;
                hipError_t ee = hipSuccess;
                if (!p->ik_ev[set]) {
                    ee = hipEventCreateWithFlags(&p->ik_ev[set], hipEventDisableTiming);
                    if (ee != hipSuccess) p->ik_ev[set] = nullptr;
                } else if (per_thread || p->ik_stream[set] != stream) {
                    wait_set = set;  // (after the lock: see below)
                }
                if (ee != hipSuccess)
                    return set_error(KIN_E_DEVICE, std::string("kin_ik_dls_batch: two-phase scratch set: ") +
                                                       hipGetErrorString(ee));
                p->ik_busy[set] = true;
                p->ik_tick[set] = ++p->ik_ticks;
                ++p->ik_stats.two_phase_calls;
            } else if (kin_plan::kIkEagerSets + p->ik_captured < kin_plan::kIkScratchSets) {
                set = kin_plan::kIkEagerSets + p->ik_captured++;
                ++p->ik_stats.captured_calls;
            } else {
                ++p->ik_stats.captured_one_phase;
            }
        }
        if (set >= 0 && !capturing) eager_set = set;
        if (wait_set >= 0) {
            // Order this call after the set's previous call on another stream (or another thread's per-thread
            // stream): nothing to do once that call has finished, else a host wait for it, outside the lock (the
            // set is ours: ik_busy).  Not hipStreamWaitEvent: on this runtime, waiting on an event last recorded
            // on a per-thread stream whose thread has since exited puts the waiting stream into a stream-capture
            // state (its later events report hipErrorCapturedEvent, legacy-stream work fails "not permitted when
            // capturing": tools/pts_probe.hip, profiles/r06_pts_probe.txt); the event itself stays valid for
            // hipEventQuery / hipEventSynchronize, and a thread's exit drains its per-thread stream (same probe).
            hipError_t ee = ik_set_state(p, wait_set, false);
            if (ee == hipErrorNotReady) {
                ee = ik_set_state(p, wait_set, true);
                std::lock_guard<std::mutex> lk(p->ik_mu);
                ++p->ik_stats.set_waits;
            }
            if (ee != hipSuccess) {
                std::lock_guard<std::mutex> lk(p->ik_mu);
                p->ik_busy[set] = false;
                p->ik_cv.notify_one();
                return set_error(KIN_E_DEVICE, std::string("kin_ik_dls_batch: two-phase scratch ordering: ") +
                                                   hipGetErrorString(ee));
            }
        }
        if (set >= 0) {  // (no set left: one phase)
            unsigned char* base = (unsigned char*)p->d_ikscr + set_bytes * set;
            scr.fail_ctl = (uint32_t*)base;
            scr.fail_list = (int32_t*)(base + ctl_bytes);
            scr.fail_aux = scr.fail_list + ring_cap * kIkSubRings;
            scr.cap = kin_plan::kIkScratchCap;
            scr.ring_cap = ring_cap;
        }
    }
    hipError_t e;
    if (p->dtype == KIN_F32)
        e = launch_ik_dls<float>(p->pf, (const KStep<float>*)p->d_steps, p->geom, a, (const float*)target, ldt,
                                 (const float*)q0, (float*)q, ldq, n, iters, (float*)err, lde, jf, scr, (hipStream_t)stream);
    else
        e = launch_ik_dls<double>(p->pd, (const KStep<double>*)p->d_steps, p->geom, a, (const double*)target, ldt,
                                  (const double*)q0, (double*)q, ldq, n, iters, (double*)err, lde, jf, scr,
                                  (hipStream_t)stream);
    if (eager_set >= 0) {  // the set's next call is ordered after this event (or after this stream's work)
        {
            std::lock_guard<std::mutex> lk(p->ik_mu);
            if (hipEventRecord(p->ik_ev[eager_set], (hipStream_t)stream) != hipSuccess)
                (void)hipStreamSynchronize((hipStream_t)stream);  // (the event then orders nothing: drain first)
            p->ik_stream[eager_set] = stream;
            p->ik_busy[eager_set] = false;
        }
        p->ik_cv.notify_one();
    }
    if (e != hipSuccess)
        return set_error(KIN_E_DEVICE, std::string("k_ik_dls launch: ") + hipGetErrorString(e) +
                                           (ik_last_call_partial() ? " (phase 2 failed to launch after phase 1: the "
                                                                     "outputs of the targets phase 1 did not solve are "
                                                                     "undefined)"
                                                                   : ""));
    return KIN_OK;
}

int kin_ik_dls_batch(const kin_plan* p, const kin_ik_params* prm, const void* target, int64_t ldt, void* q,
                     int64_t ldq, int64_t n, int32_t* iters, void* err, int64_t lde, void* stream) {
    return ik_dls_batch(p, prm, target, ldt, nullptr, q, ldq, n, iters, err, lde, stream);
}

int kin_ik_dls_batch_from(const kin_plan* p, const kin_ik_params* prm, const void* target, int64_t ldt, const void* q0,
                          void* q, int64_t ldq, int64_t n, int32_t* iters, void* err, int64_t lde, void* stream) {
    if (!q0) return set_error(KIN_E_INVALID, "kin_ik_dls_batch_from: null q0");
    return ik_dls_batch(p, prm, target, ldt, q0 == q ? nullptr : q0, q, ldq, n, iters, err, lde, stream);
}

int kin_ik_dls_batch_trace(const kin_plan* p, const kin_ik_params* prm, const void* target, int64_t ldt,
                           const void* q0, void* q, int64_t ldq, int64_t n, int32_t* iters, void* trace, int64_t ldtr,
                           void* stream) {
    if (!q0 || !trace) return set_error(KIN_E_INVALID, "kin_ik_dls_batch_trace: null q0 / trace");
    return ik_dls_batch(p, prm, target, ldt, q0 == q ? nullptr : q0, q, ldq, n, iters, nullptr, 0, stream, trace, ldtr);
}

int kin_plan_ik_sched_stats(const kin_plan* p, kin_ik_sched_stats* out) {
    if (!p || !out) return set_error(KIN_E_INVALID, "kin_plan_ik_sched_stats: null plan / out");
    std::lock_guard<std::mutex> lk(p->ik_mu);
    *out = p->ik_stats;
    return KIN_OK;
}

int kin_point_ik_nakamura_batch(const kin_plan* p, const void* pts, int64_t ldpt, void* q, int64_t ldq, int64_t n,
                                void* stream) {
    if (!p) return set_error(KIN_E_INVALID, "null plan");
    if (!p->ik_ok || p->with_base)
        return set_error(KIN_E_INVALID, "kin_point_ik_nakamura_batch: plan needs jac joints == q joints, no base");
    if (n < 0) return set_error(KIN_E_INVALID, "n < 0");
    if (n == 0) return KIN_OK;
    if (!pts || ldpt < n || !q || ldq < n) return set_error(KIN_E_INVALID, "bad pointer / stride");
    if (const int rc = check_device(p->device, "kin_point_ik_nakamura_batch", "the plan")) return rc;
    hipError_t e;
    if (p->dtype == KIN_F32)
        e = launch_nakamura<float>(p->pf, (const KStep<float>*)p->d_steps, p->geom, (const float*)pts, ldpt,
                                   (float*)q, ldq, n, jit_fns(p->jit), (hipStream_t)stream);
    else
        e = launch_nakamura<double>(p->pd, (const KStep<double>*)p->d_steps, p->geom, (const double*)pts, ldpt,
                                    (double*)q, ldq, n, jit_fns(p->jit), (hipStream_t)stream);
    if (e != hipSuccess) return set_error(KIN_E_DEVICE, std::string("k_nakamura launch: ") + hipGetErrorString(e));
    return KIN_OK;
}

}  // extern "C"
