// Internal (non-ABI) helpers shared by the C ABI translation units of libmpcfatigue.so.
#pragma once
#include <string>

#include "../../include/mpcfatigue.h"
#include "model.hpp"

namespace mf {
int capi_fail(int code, const std::string &msg);                       // sets mf_last_error()
int capi_model_dev(mf_model *m, const DevModel **dev, const Model **host);  // uploads on first use
int capi_frame_dev(mf_model *m, int frame, DevFrame **out);
int capi_ensure_device();
}  // namespace mf
