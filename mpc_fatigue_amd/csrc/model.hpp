// Kinematic-tree model shared by the URDF ingestion (host) and the kernels (device).
#pragma once
#include <string>
#include <vector>

#include "../../include/mpcfatigue.h"

namespace mf {

struct Joint {
    std::string name;
    int parent = -1;
    double R[9], t[3], axis[3];
    double mass = 0, com[3] = {0, 0, 0}, Ic[9] = {0};
    double lower, upper, effort, velocity;
};

struct Frame {
    std::string name;
    int parent = -1;
    double R[9], t[3];
};

struct Model {
    std::vector<Joint> joints;
    std::vector<Frame> frames;
    double gravity[3];
};

Model build_model_from_urdf(const char *xml);

// ---- device-side POD images -------------------------------------------------
struct DevJoint {
    double RX[9];    // placement rotation in the parent joint frame (row-major)
    double tX[3];    // placement translation
    double axis[3];  // unit joint axis (joint frame)
    double K[9];     // [axis]x
    double K2[9];    // [axis]x^2
    double m, c[3], Ic[9];
    double uX[3];    // RX^T tX: R_parent tX = A_i E_i^T uX (reverse-sweep reconstruction, adj.hpp)
    int parent;
    int pad;
};

struct DevModel {
    int n;
    int serial;      // 1 if parent[i] == i-1 for all i
    double g[3];
    DevJoint j[MF_MAX_JOINTS];
};

struct DevFrame {
    int parent;
    int pad;
    double R[9], t[3];
};

DevModel make_dev_model(const Model &M);
DevFrame make_dev_frame(const Model &M, int frame);

}  // namespace mf
