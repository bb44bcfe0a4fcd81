// kinhip_urdf.cpp -- host URDF reader (replaces parse_urdf's skrobot call,
// src/load_urdf.jl:20-80).
//
// A small XML subset parser (elements, attributes, comments, processing
// instructions, CDATA skipped; the five predefined entities decoded) and the
// URDF semantics Kinematics.jl inherits from skrobot's vendored urdfpy:
//   - link / joint ids in XML document order, 1-based (src/load_urdf.jl:22-32)
//   - <origin xyz rpy>: T = translation(xyz) * Rz(yaw) Ry(pitch) Rx(roll)
//   - <axis xyz>: default (1, 0, 0), normalised
//   - revolute / prismatic: <limit lower upper> (default 0); continuous:
//     revolute with +-Inf limits (src/load_urdf.jl:53-54); fixed;
//     anything else -> KIN_E_PARSE (src/load_urdf.jl:62 throw(Exception))
//   - BoxMetaData from the first box <collision> (src/load_urdf.jl:1-18)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "kinhip.h"
#include "kinhip_host.h"

namespace {

struct XNode {
    std::string tag;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<std::unique_ptr<XNode>> kids;
    const std::string* attr(const char* k) const {
        for (auto& a : attrs)
            if (a.first == k) return &a.second;
        return nullptr;
    }
    const XNode* child(const char* t) const {
        for (auto& k : kids)
            if (k->tag == t) return k.get();
        return nullptr;
    }
};

struct XParser {
    const char* p;
    const char* e;
    std::string err;

    bool fail(const char* msg) {
        if (err.empty()) err = msg;
        return false;
    }
    void ws() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
    }
    bool starts(const char* s) const {
        size_t n = strlen(s);
        return (size_t)(e - p) >= n && memcmp(p, s, n) == 0;
    }
    bool skip_until(const char* s) {
        size_t n = strlen(s);
        while ((size_t)(e - p) >= n) {
            if (memcmp(p, s, n) == 0) {
                p += n;
                return true;
            }
            ++p;
        }
        return fail("unterminated markup");
    }
    static std::string decode(const std::string& s) {
        std::string o;
        for (size_t i = 0; i < s.size(); ++i) {
            if (s[i] == '&') {
                static const char* ent[5][2] = {{"&lt;", "<"}, {"&gt;", ">"}, {"&amp;", "&"}, {"&quot;", "\""}, {"&apos;", "'"}};
                bool hit = false;
                for (auto& en : ent) {
                    size_t n = strlen(en[0]);
                    if (s.compare(i, n, en[0]) == 0) {
                        o += en[1];
                        i += n - 1;
                        hit = true;
                        break;
                    }
                }
                if (!hit) o += s[i];
            } else {
                o += s[i];
            }
        }
        return o;
    }
    // skip text, comments, PIs, doctype, CDATA until the next element tag
    bool misc() {
        for (;;) {
            while (p < e && *p != '<') ++p;
            if (p >= e) return true;
            if (starts("<!--")) { if (!skip_until("-->")) return false; continue; }
            if (starts("<?")) { if (!skip_until("?>")) return false; continue; }
            if (starts("<![CDATA[")) { if (!skip_until("]]>")) return false; continue; }
            if (starts("<!")) { if (!skip_until(">")) return false; continue; }
            return true;
        }
    }
    bool name(std::string& out) {
        const char* s = p;
        while (p < e && (isalnum((unsigned char)*p) || *p == '_' || *p == '-' || *p == ':' || *p == '.')) ++p;
        if (p == s) return fail("expected a name");
        out.assign(s, p);
        return true;
    }
    // parses one element starting at '<'
    bool element(XNode& n) {
        ++p;  // '<'
        if (!name(n.tag)) return false;
        for (;;) {
            ws();
            if (p >= e) return fail("unexpected end in tag");
            if (*p == '/') {
                if (p + 1 >= e || p[1] != '>') return fail("bad empty-element tag");
                p += 2;
                return true;
            }
            if (*p == '>') {
                ++p;
                break;
            }
            std::string k;
            if (!name(k)) return false;
            ws();
            if (p >= e || *p != '=') return fail("expected '='");
            ++p;
            ws();
            if (p >= e || (*p != '"' && *p != '\'')) return fail("expected a quoted value");
            char qch = *p++;
            const char* s = p;
            while (p < e && *p != qch) ++p;
            if (p >= e) return fail("unterminated attribute");
            n.attrs.emplace_back(k, decode(std::string(s, p)));
            ++p;
        }
        for (;;) {
            if (!misc()) return false;
            if (p >= e) return fail("unterminated element");
            if (starts("</")) {
                p += 2;
                std::string t;
                if (!name(t)) return false;
                if (t != n.tag) return fail("mismatched closing tag");
                ws();
                if (p >= e || *p != '>') return fail("bad closing tag");
                ++p;
                return true;
            }
            auto kid = std::make_unique<XNode>();
            if (!element(*kid)) return false;
            n.kids.push_back(std::move(kid));
        }
    }
};

bool parse_vec(const std::string* s, int n, double* out, std::string& err) {
    if (!s) return false;
    const char* c = s->c_str();
    for (int k = 0; k < n; ++k) {
        char* end;
        out[k] = strtod(c, &end);
        if (end == c) {
            err = "malformed number list '" + *s + "'";
            return false;
        }
        c = end;
    }
    return true;
}

// urdfpy rpy_to_matrix: Rz(y) Ry(p) Rx(r); column-major 4x4 with translation
bool origin_tf(const XNode* o, double* T16, std::string& err) {
    double xyz[3] = {0, 0, 0}, rpy[3] = {0, 0, 0};
    if (o) {
        if (const std::string* s = o->attr("xyz"))
            if (!parse_vec(s, 3, xyz, err)) return false;
        if (const std::string* s = o->attr("rpy"))
            if (!parse_vec(s, 3, rpy, err)) return false;
    }
    const double c3 = cos(rpy[0]), c2 = cos(rpy[1]), c1 = cos(rpy[2]);
    const double s3 = sin(rpy[0]), s2 = sin(rpy[1]), s1 = sin(rpy[2]);
    const double R[3][3] = {{c1 * c2, (c1 * s2 * s3) - (c3 * s1), (s1 * s3) + (c1 * c3 * s2)},
                            {c2 * s1, (c1 * c3) + (s1 * s2 * s3), (c3 * s1 * s2) - (c1 * s3)},
                            {-s2, c2 * s3, c2 * c3}};
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) T16[i + 4 * j] = (i == j) ? 1.0 : 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) T16[i + 4 * j] = R[i][j];
    for (int i = 0; i < 3; ++i) T16[i + 12] = xyz[i];
    return true;
}

}  // namespace

struct kin_urdf {
    std::string robot_name;
    std::vector<std::string> link_names, joint_names;
    std::unordered_map<std::string, int32_t> link_id, joint_id;
    std::vector<int32_t> jtype, jplink, jclink;
    std::vector<double> jpose, jaxis, jlo, jhi;
    std::vector<int32_t> has_box;
    std::vector<double> box_ext, box_origin;
};

static int parse_doc(const char* xml, size_t len, kin_urdf** out) {
    using namespace kinhip;
    if (!xml || !out) return set_error(KIN_E_INVALID, "kin_urdf_parse: null argument");
    XParser ps{xml, xml + len, {}};
    if (!ps.misc() || ps.p >= ps.e) return set_error(KIN_E_PARSE, "URDF: no root element " + ps.err);
    XNode root;
    if (!ps.element(root)) return set_error(KIN_E_PARSE, "URDF: XML error: " + ps.err);
    if (root.tag != "robot") return set_error(KIN_E_PARSE, "URDF: root element is <" + root.tag + ">, not <robot>");
    auto u = std::make_unique<kin_urdf>();
    if (auto* n = root.attr("name")) u->robot_name = *n;
    std::string err;
    for (auto& k : root.kids) {
        if (k->tag != "link") continue;
        const std::string* nm = k->attr("name");
        if (!nm) return set_error(KIN_E_PARSE, "URDF: <link> without a name");
        const int32_t id = (int32_t)u->link_names.size() + 1;
        u->link_names.push_back(*nm);
        u->link_id[*nm] = id;
        double ext[3] = {0, 0, 0}, org[16];
        int32_t hb = 0;
        origin_tf(nullptr, org, err);
        for (auto& c : k->kids) {
            if (c->tag != "collision") continue;
            const XNode* g = c->child("geometry");
            const XNode* b = g ? g->child("box") : nullptr;
            if (!b) continue;
            if (!parse_vec(b->attr("size"), 3, ext, err) || !origin_tf(c->child("origin"), org, err))
                return set_error(KIN_E_PARSE, "URDF: link " + *nm + ": " + err);
            hb = 1;
            break;
        }
        u->has_box.push_back(hb);
        u->box_ext.insert(u->box_ext.end(), ext, ext + 3);
        u->box_origin.insert(u->box_origin.end(), org, org + 16);
    }
    for (auto& k : root.kids) {
        if (k->tag != "joint") continue;
        const std::string* nm = k->attr("name");
        const std::string* ty = k->attr("type");
        if (!nm || !ty) return set_error(KIN_E_PARSE, "URDF: <joint> without name/type");
        const XNode* par = k->child("parent");
        const XNode* chd = k->child("child");
        const std::string* pl = par ? par->attr("link") : nullptr;
        const std::string* cl = chd ? chd->attr("link") : nullptr;
        if (!pl || !cl) return set_error(KIN_E_PARSE, "URDF: joint " + *nm + " lacks parent/child");
        auto ip = u->link_id.find(*pl), ic = u->link_id.find(*cl);
        if (ip == u->link_id.end() || ic == u->link_id.end())
            return set_error(KIN_E_KEY, "URDF: joint " + *nm + " refers to an unknown link");
        int32_t t;
        double lo = -INFINITY, hi = INFINITY;
        const XNode* lim = k->child("limit");
        auto limits = [&]() {
            lo = 0.0;
            hi = 0.0;
            if (lim) {
                if (auto* s = lim->attr("lower")) lo = strtod(s->c_str(), nullptr);
                if (auto* s = lim->attr("upper")) hi = strtod(s->c_str(), nullptr);
            }
        };
        if (*ty == "revolute") { t = KIN_JOINT_REVOLUTE; limits(); }
        else if (*ty == "continuous") { t = KIN_JOINT_REVOLUTE; }
        else if (*ty == "prismatic") { t = KIN_JOINT_PRISMATIC; limits(); }
        else if (*ty == "fixed") { t = KIN_JOINT_FIXED; }
        else return set_error(KIN_E_PARSE, "URDF: joint " + *nm + " has unsupported type '" + *ty + "'");
        double T16[16];
        if (!origin_tf(k->child("origin"), T16, err)) return set_error(KIN_E_PARSE, "URDF: joint " + *nm + ": " + err);
        double ax[3] = {1, 0, 0};
        if (const XNode* a = k->child("axis")) {
            if (!parse_vec(a->attr("xyz"), 3, ax, err)) return set_error(KIN_E_PARSE, "URDF: joint " + *nm + ": " + err);
            const double nn = sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
            if (nn > 0)
                for (double& v : ax) v /= nn;
        }
        const int32_t id = (int32_t)u->joint_names.size() + 1;
        u->joint_names.push_back(*nm);
        u->joint_id[*nm] = id;
        u->jtype.push_back(t);
        u->jplink.push_back(ip->second);
        u->jclink.push_back(ic->second);
        u->jpose.insert(u->jpose.end(), T16, T16 + 16);
        u->jaxis.insert(u->jaxis.end(), ax, ax + 3);
        u->jlo.push_back(lo);
        u->jhi.push_back(hi);
    }
    *out = u.release();
    return KIN_OK;
}

extern "C" {

int kin_urdf_parse_string(const char* xml, size_t len, kin_urdf** out) { return parse_doc(xml, len, out); }

int kin_urdf_parse_file(const char* path, kin_urdf** out) {
    if (!path) return kinhip::set_error(KIN_E_INVALID, "kin_urdf_parse_file: null path");
    std::ifstream f(path, std::ios::binary);
    if (!f) return kinhip::set_error(KIN_E_IO, std::string("cannot open ") + path);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string s = ss.str();
    return parse_doc(s.data(), s.size(), out);
}

int kin_urdf_destroy(kin_urdf* u) {
    delete u;
    return KIN_OK;
}

int kin_urdf_tree(const kin_urdf* u, int32_t with_base, kin_tree_desc* d) {
    if (!u || !d) return kinhip::set_error(KIN_E_INVALID, "kin_urdf_tree: null argument");
    d->n_links = (int32_t)u->link_names.size();
    d->n_joints = (int32_t)u->joint_names.size();
    d->joint_type = u->jtype.data();
    d->joint_plink = u->jplink.data();
    d->joint_clink = u->jclink.data();
    d->joint_pose = u->jpose.data();
    d->joint_axis = u->jaxis.data();
    d->joint_lower = u->jlo.data();
    d->joint_upper = u->jhi.data();
    d->with_base = with_base ? 1 : 0;
    return KIN_OK;
}

int kin_urdf_link_name(const kin_urdf* u, int32_t id, const char** name) {
    if (!u || !name) return kinhip::set_error(KIN_E_INVALID, "null argument");
    if (id < 1 || id > (int32_t)u->link_names.size()) return kinhip::set_error(KIN_E_KEY, "link id out of range");
    *name = u->link_names[id - 1].c_str();
    return KIN_OK;
}

int kin_urdf_joint_name(const kin_urdf* u, int32_t id, const char** name) {
    if (!u || !name) return kinhip::set_error(KIN_E_INVALID, "null argument");
    if (id < 1 || id > (int32_t)u->joint_names.size()) return kinhip::set_error(KIN_E_KEY, "joint id out of range");
    *name = u->joint_names[id - 1].c_str();
    return KIN_OK;
}

int kin_urdf_find_link(const kin_urdf* u, const char* name, int32_t* id) {
    if (!u || !name || !id) return kinhip::set_error(KIN_E_INVALID, "null argument");
    auto it = u->link_id.find(name);
    if (it == u->link_id.end()) return kinhip::set_error(KIN_E_KEY, std::string("KeyError: link ") + name);
    *id = it->second;
    return KIN_OK;
}

int kin_urdf_find_joint(const kin_urdf* u, const char* name, int32_t* id) {
    if (!u || !name || !id) return kinhip::set_error(KIN_E_INVALID, "null argument");
    auto it = u->joint_id.find(name);
    if (it == u->joint_id.end()) return kinhip::set_error(KIN_E_KEY, std::string("KeyError: joint ") + name);
    *id = it->second;
    return KIN_OK;
}

int kin_urdf_link_box(const kin_urdf* u, int32_t id, int32_t* has_box, double* ext3, double* org16) {
    if (!u || !has_box) return kinhip::set_error(KIN_E_INVALID, "null argument");
    if (id < 1 || id > (int32_t)u->link_names.size()) return kinhip::set_error(KIN_E_KEY, "link id out of range");
    *has_box = u->has_box[id - 1];
    if (ext3) memcpy(ext3, &u->box_ext[3 * (id - 1)], sizeof(double) * 3);
    if (org16) memcpy(org16, &u->box_origin[16 * (id - 1)], sizeof(double) * 16);
    return KIN_OK;
}

}  // extern "C"
