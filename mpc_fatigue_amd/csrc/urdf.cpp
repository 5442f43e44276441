// URDF -> kinematic-tree model with Pinocchio semantics (host code of libmpcfatigue.so).
//
// Replaces urdf::parseURDF + pinocchio::urdf::buildModel(urdf, model, true) as
// called at src/casadi_pinocchio_bridge.hpp:60-63 (fixed base, no root joint):
//   * one root link attached to the universe (its inertia never moves);
//   * revolute joints become 1-DoF joints, placement = (placement of the parent
//     link in its joint frame) * origin(joint);
//   * children of fixed joints are merged into the parent joint body (inertia
//     appended with the accumulated placement; link name becomes a BODY frame);
//   * child joints are visited in joint-name order (urdfdom keeps them in a
//     std::map), depth first;
//   * rpy = Rz(y) Ry(p) Rx(r); inertial origin rpy rotates the tensor.
// Only what the hot path needs is parsed: links, joints, origins, axes,
// limits, inertials.  Continuous / prismatic / floating joints -> error.
#include "model.hpp"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace mf {

namespace {

struct XNode {
    std::string tag;
    std::map<std::string, std::string> attr;
    std::vector<std::unique_ptr<XNode>> kids;
    const XNode *child(const char *t) const {
        for (auto &k : kids)
            if (k->tag == t) return k.get();
        return nullptr;
    }
    const char *get(const char *a) const {
        auto it = attr.find(a);
        return it == attr.end() ? nullptr : it->second.c_str();
    }
};

// Minimal XML reader: elements, attributes, comments, declarations; text is ignored.
struct XReader {
    const char *s;
    size_t i = 0, n;
    explicit XReader(const char *src) : s(src), n(strlen(src)) {}
    [[noreturn]] void fail(const char *what) {
        throw std::runtime_error(std::string("URDF parse error: ") + what + " at byte " + std::to_string(i));
    }
    void ws() {
        while (i < n && isspace((unsigned char)s[i])) i++;
    }
    bool starts(const char *p) const { return strncmp(s + i, p, strlen(p)) == 0; }
    void skip_misc() {
        for (;;) {
            while (i < n && s[i] != '<') i++;
            if (i >= n) return;
            if (starts("<!--")) {
                const char *e = strstr(s + i + 4, "-->");
                if (!e) fail("unterminated comment");
                i = (size_t)(e - s) + 3;
            } else if (starts("<?") || starts("<!")) {
                const char *e = strchr(s + i, '>');
                if (!e) fail("unterminated declaration");
                i = (size_t)(e - s) + 1;
            } else {
                return;
            }
        }
    }
    std::string name() {
        size_t b = i;
        while (i < n && (isalnum((unsigned char)s[i]) || s[i] == '_' || s[i] == ':' || s[i] == '-' || s[i] == '.')) i++;
        if (b == i) fail("expected name");
        return std::string(s + b, i - b);
    }
    std::unique_ptr<XNode> element() {
        skip_misc();
        if (i >= n || s[i] != '<') fail("expected element");
        i++;
        auto nd = std::make_unique<XNode>();
        nd->tag = name();
        for (;;) {
            ws();
            if (i >= n) fail("unterminated tag");
            if (s[i] == '/') {
                if (i + 1 >= n || s[i + 1] != '>') fail("bad self-closing tag");
                i += 2;
                return nd;
            }
            if (s[i] == '>') { i++; break; }
            std::string a = name();
            ws();
            if (i >= n || s[i] != '=') fail("expected '='");
            i++;
            ws();
            char q = s[i];
            if (q != '"' && q != '\'') fail("expected quote");
            size_t b = ++i;
            while (i < n && s[i] != q) i++;
            if (i >= n) fail("unterminated attribute");
            nd->attr[a] = std::string(s + b, i - b);
            i++;
        }
        for (;;) {
            // skip text and comments until the next tag
            for (;;) {
                while (i < n && s[i] != '<') i++;
                if (i >= n) fail("unterminated element");
                if (starts("<!--")) {
                    const char *e = strstr(s + i + 4, "-->");
                    if (!e) fail("unterminated comment");
                    i = (size_t)(e - s) + 3;
                    continue;
                }
                break;
            }
            if (starts("</")) {
                i += 2;
                std::string t = name();
                if (t != nd->tag) fail("mismatched closing tag");
                ws();
                if (i >= n || s[i] != '>') fail("expected '>'");
                i++;
                return nd;
            }
            nd->kids.push_back(element());
        }
    }
};

struct V3 { double x[3]; };
struct M3 { double a[9]; };

M3 mul(const M3 &A, const M3 &B) {
    M3 C;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) C.a[3 * r + c] = A.a[3 * r] * B.a[c] + A.a[3 * r + 1] * B.a[3 + c] + A.a[3 * r + 2] * B.a[6 + c];
    return C;
}
V3 mulv(const M3 &A, const V3 &v) {
    V3 o;
    for (int r = 0; r < 3; r++) o.x[r] = A.a[3 * r] * v.x[0] + A.a[3 * r + 1] * v.x[1] + A.a[3 * r + 2] * v.x[2];
    return o;
}
M3 transpose(const M3 &A) {
    M3 T;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) T.a[3 * r + c] = A.a[3 * c + r];
    return T;
}
M3 eye() { return M3{{1, 0, 0, 0, 1, 0, 0, 0, 1}}; }
M3 rpy(double r, double p, double y) {
    double cr = cos(r), sr = sin(r), cp = cos(p), sp = sin(p), cy = cos(y), sy = sin(y);
    M3 Rx{{1, 0, 0, 0, cr, -sr, 0, sr, cr}}, Ry{{cp, 0, sp, 0, 1, 0, -sp, 0, cp}}, Rz{{cy, -sy, 0, sy, cy, 0, 0, 0, 1}};
    return mul(Rz, mul(Ry, Rx));
}
V3 parse3(const char *s, V3 def) {
    if (!s) return def;
    V3 v;
    char *e = nullptr;
    for (int k = 0; k < 3; k++) {
        v.x[k] = strtod(s, &e);
        if (e == s) throw std::runtime_error("URDF: bad 3-vector '" + std::string(s) + "'");
        s = e;
    }
    return v;
}
double attrd(const XNode *nd, const char *a, double def) {
    const char *s = nd ? nd->get(a) : nullptr;
    return s ? strtod(s, nullptr) : def;
}

struct Inertia {
    double m = 0;
    V3 c{{0, 0, 0}};
    M3 I{{0, 0, 0, 0, 0, 0, 0, 0, 0}};
};
Inertia transformed(const Inertia &in, const M3 &R, const V3 &t) {
    Inertia o;
    o.m = in.m;
    V3 rc = mulv(R, in.c);
    for (int k = 0; k < 3; k++) o.c.x[k] = rc.x[k] + t.x[k];
    o.I = mul(R, mul(in.I, transpose(R)));
    return o;
}
Inertia combine(const Inertia &a, const Inertia &b) {
    Inertia o;
    o.m = a.m + b.m;
    if (o.m <= 0) return Inertia();
    for (int k = 0; k < 3; k++) o.c.x[k] = (a.m * a.c.x[k] + b.m * b.c.x[k]) / o.m;
    auto shift = [&](const Inertia &X) {
        M3 S = X.I;
        double d[3] = {X.c.x[0] - o.c.x[0], X.c.x[1] - o.c.x[1], X.c.x[2] - o.c.x[2]};
        double dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) S.a[3 * r + c] += X.m * ((r == c ? dd : 0.0) - d[r] * d[c]);
        return S;
    };
    M3 A = shift(a), B = shift(b);
    for (int k = 0; k < 9; k++) o.I.a[k] = A.a[k] + B.a[k];
    return o;
}

}  // namespace

Model build_model_from_urdf(const char *xml) {
    XReader rd(xml);
    std::unique_ptr<XNode> robot = rd.element();
    if (robot->tag != "robot") throw std::runtime_error("URDF: root element is not <robot>");
    std::map<std::string, const XNode *> links;
    std::vector<const XNode *> joints;
    for (auto &k : robot->kids) {
        if (k->tag == "link") {
            const char *nm = k->get("name");
            if (!nm) throw std::runtime_error("URDF: link without name");
            links[nm] = k.get();
        } else if (k->tag == "joint") {
            joints.push_back(k.get());
        }
    }
    std::sort(joints.begin(), joints.end(), [](const XNode *a, const XNode *b) {
        return std::string(a->get("name") ? a->get("name") : "") < std::string(b->get("name") ? b->get("name") : "");
    });
    std::map<std::string, std::vector<const XNode *>> child_of;
    std::map<std::string, bool> has_parent;
    for (const XNode *j : joints) {
        const XNode *p = j->child("parent"), *c = j->child("child");
        if (!p || !c || !p->get("link") || !c->get("link")) throw std::runtime_error("URDF: joint without parent/child");
        child_of[p->get("link")].push_back(j);
        has_parent[c->get("link")] = true;
    }
    std::vector<std::string> roots;
    for (auto &kv : links)
        if (!has_parent.count(kv.first)) roots.push_back(kv.first);
    if (roots.size() != 1) throw std::runtime_error("URDF: expected exactly one root link");

    auto link_inertia = [&](const std::string &name) {
        Inertia I;
        auto it = links.find(name);
        if (it == links.end()) throw std::runtime_error("URDF: joint refers to unknown link " + name);
        const XNode *in = it->second->child("inertial");
        if (!in) return I;
        const XNode *o = in->child("origin");
        V3 xyz = parse3(o ? o->get("xyz") : nullptr, V3{{0, 0, 0}});
        V3 r = parse3(o ? o->get("rpy") : nullptr, V3{{0, 0, 0}});
        I.m = attrd(in->child("mass"), "value", 0.0);
        const XNode *ie = in->child("inertia");
        double ixx = attrd(ie, "ixx", 0), ixy = attrd(ie, "ixy", 0), ixz = attrd(ie, "ixz", 0);
        double iyy = attrd(ie, "iyy", 0), iyz = attrd(ie, "iyz", 0), izz = attrd(ie, "izz", 0);
        M3 Iu{{ixx, ixy, ixz, ixy, iyy, iyz, ixz, iyz, izz}};
        M3 R = rpy(r.x[0], r.x[1], r.x[2]);
        I.c = xyz;
        I.I = mul(R, mul(Iu, transpose(R)));
        return I;
    };

    Model M;
    M.gravity[0] = 0; M.gravity[1] = 0; M.gravity[2] = -9.81;
    std::vector<Inertia> body;
    auto add_frame = [&](const std::string &nm, int parent, const M3 &R, const V3 &t) {
        for (auto &f : M.frames)
            if (f.name == nm) return;
        Frame f;
        f.name = nm;
        f.parent = parent;
        memcpy(f.R, R.a, sizeof f.R);
        memcpy(f.t, t.x, sizeof f.t);
        M.frames.push_back(f);
    };
    add_frame(roots[0], -1, eye(), V3{{0, 0, 0}});

    std::function<void(const std::string &, int, const M3 &, const V3 &)> visit;
    visit = [&](const std::string &link, int pj, const M3 &Rl, const V3 &tl) {
        for (const XNode *j : child_of[link]) {
            const XNode *o = j->child("origin");
            V3 xyz = parse3(o ? o->get("xyz") : nullptr, V3{{0, 0, 0}});
            V3 r = parse3(o ? o->get("rpy") : nullptr, V3{{0, 0, 0}});
            M3 Rj = mul(Rl, rpy(r.x[0], r.x[1], r.x[2]));
            V3 tj = mulv(Rl, xyz);
            for (int k = 0; k < 3; k++) tj.x[k] += tl.x[k];
            std::string child = j->child("child")->get("link");
            std::string jt = j->get("type") ? j->get("type") : "";
            std::string jn = j->get("name") ? j->get("name") : "";
            if (jt == "fixed") {
                add_frame(jn, pj, Rj, tj);
                add_frame(child, pj, Rj, tj);
                if (pj >= 0) body[pj] = combine(body[pj], transformed(link_inertia(child), Rj, tj));
                visit(child, pj, Rj, tj);
            } else if (jt == "revolute") {
                if ((int)M.joints.size() >= MF_MAX_JOINTS) throw std::runtime_error("URDF: too many joints");
                const XNode *ax = j->child("axis");
                V3 a = parse3(ax ? ax->get("xyz") : nullptr, V3{{1, 0, 0}});
                double na = sqrt(a.x[0] * a.x[0] + a.x[1] * a.x[1] + a.x[2] * a.x[2]);
                if (!(na > 0)) throw std::runtime_error("URDF: zero joint axis");
                Joint J;
                J.name = jn;
                J.parent = pj;
                memcpy(J.R, Rj.a, sizeof J.R);
                memcpy(J.t, tj.x, sizeof J.t);
                for (int k = 0; k < 3; k++) J.axis[k] = a.x[k] / na;
                const XNode *lim = j->child("limit");
                J.lower = attrd(lim, "lower", -INFINITY);
                J.upper = attrd(lim, "upper", INFINITY);
                J.effort = attrd(lim, "effort", INFINITY);
                J.velocity = attrd(lim, "velocity", INFINITY);
                int idx = (int)M.joints.size();
                M.joints.push_back(J);
                body.push_back(link_inertia(child));
                add_frame(jn, idx, eye(), V3{{0, 0, 0}});
                add_frame(child, idx, eye(), V3{{0, 0, 0}});
                visit(child, idx, eye(), V3{{0, 0, 0}});
            } else {
                throw std::runtime_error("URDF: unsupported joint type '" + jt + "' (joint " + jn + ")");
            }
        }
    };
    visit(roots[0], -1, eye(), V3{{0, 0, 0}});
    for (size_t k = 0; k < M.joints.size(); k++) {
        M.joints[k].mass = body[k].m;
        memcpy(M.joints[k].com, body[k].c.x, sizeof M.joints[k].com);
        memcpy(M.joints[k].Ic, body[k].I.a, sizeof M.joints[k].Ic);
    }
    if (M.joints.empty()) throw std::runtime_error("URDF: no movable joints");
    return M;
}

// Device image of the model: joint placements, Rodrigues matrices K = [a]x and
// K^2 (R(q) = I + sin q K + (1 - cos q) K^2), inertial parameters.
DevModel make_dev_model(const Model &M) {
    DevModel D;
    memset(&D, 0, sizeof D);
    D.n = (int)M.joints.size();
    D.serial = 1;
    for (int k = 0; k < 3; k++) D.g[k] = M.gravity[k];
    for (int i = 0; i < D.n; i++) {
        const Joint &J = M.joints[i];
        DevJoint &d = D.j[i];
        memcpy(d.RX, J.R, sizeof d.RX);
        memcpy(d.tX, J.t, sizeof d.tX);
        memcpy(d.axis, J.axis, sizeof d.axis);
        const double *a = J.axis;
        double K[9] = {0, -a[2], a[1], a[2], 0, -a[0], -a[1], a[0], 0};
        memcpy(d.K, K, sizeof K);
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) d.K2[3 * r + c] = K[3 * r] * K[c] + K[3 * r + 1] * K[3 + c] + K[3 * r + 2] * K[6 + c];
        d.m = J.mass;
        memcpy(d.c, J.com, sizeof d.c);
        memcpy(d.Ic, J.Ic, sizeof d.Ic);
        for (int r = 0; r < 3; r++) d.uX[r] = J.R[r] * J.t[0] + J.R[3 + r] * J.t[1] + J.R[6 + r] * J.t[2];
        d.parent = J.parent;
        if (J.parent != i - 1) D.serial = 0;
    }
    return D;
}

DevFrame make_dev_frame(const Model &M, int frame) {
    DevFrame F;
    memset(&F, 0, sizeof F);
    const Frame &f = M.frames[frame];
    F.parent = f.parent;
    memcpy(F.R, f.R, sizeof F.R);
    memcpy(F.t, f.t, sizeof F.t);
    return F;
}

}  // namespace mf
