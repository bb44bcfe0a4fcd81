// Host sanitizer harness (test infrastructure; tests/test_host_sanitizers.py): drives the engine's
// host code -- the URDF reader (kinhip_urdf.cpp), tree validation, rptable, add_link and plan staging
// (kinhip_host.cpp) -- under ASan + UBSan, on the given URDF files and on seeded corruptions of them.
//   kin_host_harness [--mutants K] [--seed S] file.urdf ...
// Exit 0 when every call returned a kin_status (no crash, no sanitizer report); prints a summary.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "kinhip.h"

namespace {

uint64_t g_state = 0x9E3779B97F4A7C15ull;
uint64_t rnd() {  // splitmix64
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
double urand(double lo, double hi) { return lo + (hi - lo) * (double)(rnd() >> 11) * (1.0 / 9007199254740992.0); }

int n_parsed = 0, n_rejected = 0, n_plans = 0, n_plan_rc[16] = {};

void check_rc(int rc, const char* what) {
    if (rc > 0 || rc < -8) {
        fprintf(stderr, "%s: unexpected status %d\n", what, rc);
        abort();
    }
    (void)kin_last_error();
}

void exercise_model(kin_model* m, int with_base) {
    int32_t nl = 0, nj = 0;
    check_rc(kin_model_num_links(m, &nl), "num_links");
    check_rc(kin_model_num_joints(m, &nj), "num_joints");
    std::vector<double> ang(nj);
    for (auto& a : ang) a = urand(-3, 3);
    check_rc(kin_model_set_angles(m, ang.data()), "set_angles");
    int32_t rel = 0;
    for (int32_t j = 0; j <= nj + 1; ++j)
        for (int32_t l = 0; l <= nl + 1; ++l) check_rc(kin_model_is_relevant(m, j, l, &rel), "is_relevant");
    double T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0.1, -0.2, 0.3, 1};
    int32_t nid = 0;
    for (int k = 0; k < 3; ++k) check_rc(kin_model_add_link(m, (int32_t)(rnd() % (nl + 2)), T, &nid), "add_link");
    check_rc(kin_model_num_links(m, &nl), "num_links");
    check_rc(kin_model_num_joints(m, &nj), "num_joints");
    // plans over every link, random joint subsets (ids occasionally out of range / repeated)
    for (int32_t l = 0; l <= nl + 1; ++l) {
        std::vector<int32_t> q, out{l};
        for (int32_t j = 1; j <= nj; ++j)
            if (rnd() % 3) q.push_back(j);
        if (rnd() % 8 == 0) q.push_back((int32_t)(rnd() % (nj + 3)));  // maybe bogus / repeated
        const uint32_t flags = (uint32_t)(rnd() % 8);
        for (int dt = 0; dt < 2; ++dt) {
            kin_plan_desc d{dt, (int32_t)q.size(), q.data(), (int32_t)out.size(), out.data(),
                            (rnd() % 2) ? l : 0, (int32_t)q.size(), q.data(), flags};
            kin_plan* p = nullptr;
            const int rc = kin_plan_create(m, &d, &p);
            check_rc(rc, "plan_create");
            n_plan_rc[-rc]++;
            ++n_plans;
            if (rc == KIN_OK) {
                int32_t a, b, c;
                check_rc(kin_plan_shape(p, &a, &b, &c), "plan_shape");
                kin_plan_destroy(p);
            }
        }
        // collision plan: spheres on this link and a random one
        int32_t sl[2] = {l, (int32_t)(rnd() % (nl + 1)) + 1};
        double cen[6] = {0.01, 0, 0, 0, 0.02, 0}, rad[2] = {0.05, 0.04};
        kin_coll_desc c{(int32_t)(rnd() % 2), (int32_t)q.size(), q.data(), 2, sl, cen, rad};
        kin_plan* cp = nullptr;
        const int rc = kin_coll_plan_create(m, &c, &cp);
        check_rc(rc, "coll_plan_create");
        if (rc == KIN_OK) kin_plan_destroy(cp);
        // collision-aware IK plan: the tree of this link and the spheres (host staging runs before any
        // device allocation)
        kin_plan* ip = nullptr;
        const int rc2 = kin_coll_ik_plan_create(m, &c, (int32_t)(rnd() % (nl + 2)), &ip);
        check_rc(rc2, "coll_ik_plan_create");
        if (rc2 == KIN_OK) kin_plan_destroy(ip);
    }
    (void)with_base;
}

void exercise_text(const std::string& text) {
    kin_urdf* u = nullptr;
    int rc = kin_urdf_parse_string(text.data(), text.size(), &u);
    check_rc(rc, "parse");
    if (rc != KIN_OK) {
        ++n_rejected;
        return;
    }
    ++n_parsed;
    for (int wb = 0; wb < 2; ++wb) {
        kin_tree_desc d{};
        rc = kin_urdf_tree(u, wb, &d);
        check_rc(rc, "tree");
        if (rc != KIN_OK) continue;
        const char* nm = nullptr;
        int32_t id = 0, has = 0;
        double ext[3], org[16];
        for (int32_t l = 0; l <= d.n_links + 1; ++l) {
            if (kin_urdf_link_name(u, l, &nm) == KIN_OK) check_rc(kin_urdf_find_link(u, nm, &id), "find_link");
            check_rc(kin_urdf_link_box(u, l, &has, ext, org), "link_box");
        }
        for (int32_t j = 0; j <= d.n_joints + 1; ++j)
            if (kin_urdf_joint_name(u, j, &nm) == KIN_OK) check_rc(kin_urdf_find_joint(u, nm, &id), "find_joint");
        check_rc(kin_urdf_find_link(u, "no such link", &id), "find_link");
        kin_model* m = nullptr;
        rc = kin_model_create(&d, &m);
        check_rc(rc, "model_create");
        if (rc == KIN_OK) {
            exercise_model(m, wb);
            kin_model_destroy(m);
        }
    }
    kin_urdf_destroy(u);
}

std::string mutate(const std::string& s) {
    std::string t = s;
    static const char sig[] = "<>\"'=/&;!?- \n0.e";
    switch (rnd() % 5) {
        case 0:  // truncate
            t.resize(rnd() % (t.size() + 1));
            break;
        case 1:  // flip bytes to XML-significant characters
            for (int k = 0, n = 1 + (int)(rnd() % 8); k < n && !t.empty(); ++k) t[rnd() % t.size()] = sig[rnd() % (sizeof sig - 1)];
            break;
        case 2: {  // delete a span
            if (t.empty()) break;
            size_t a = rnd() % t.size(), b = a + rnd() % 64;
            t.erase(a, b - a);
            break;
        }
        case 3: {  // duplicate a span
            if (t.empty()) break;
            size_t a = rnd() % t.size(), n = rnd() % 256;
            t.insert(rnd() % t.size(), t.substr(a, n));
            break;
        }
        default:  // random bytes
            for (int k = 0, n = 1 + (int)(rnd() % 4); k < n && !t.empty(); ++k) t[rnd() % t.size()] = (char)(rnd() & 0xff);
    }
    return t;
}

}  // namespace

int main(int argc, char** argv) {
    int mutants = 0;
    std::vector<std::string> files;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--mutants") && i + 1 < argc) mutants = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--seed") && i + 1 < argc) g_state = strtoull(argv[++i], nullptr, 10);
        else files.push_back(argv[i]);
    }
    for (const auto& f : files) {
        std::ifstream in(f, std::ios::binary);
        if (!in) {
            fprintf(stderr, "cannot read %s\n", f.c_str());
            return 2;
        }
        std::stringstream ss;
        ss << in.rdbuf();
        const std::string text = ss.str();
        exercise_text(text);
        for (int k = 0; k < mutants; ++k) exercise_text(mutate(text));
        kin_urdf* u = nullptr;
        check_rc(kin_urdf_parse_file(f.c_str(), &u), "parse_file");
        if (u) kin_urdf_destroy(u);
    }
    check_rc(kin_model_create(nullptr, nullptr), "model_create(null)");
    printf("parsed %d rejected %d plans %d (rc: ok %d invalid %d key %d method %d device %d unsupported %d)\n",
           n_parsed, n_rejected, n_plans, n_plan_rc[0], n_plan_rc[1], n_plan_rc[2], n_plan_rc[3], n_plan_rc[4],
           n_plan_rc[5]);
    return 0;
}
