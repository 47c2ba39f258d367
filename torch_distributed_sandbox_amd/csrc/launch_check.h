// Binding-layer side of TDS_LAUNCH_CHECK (kernels/common.h): every op that launches kernels
// calls check_launches(op) before returning, which raises if any launch of the calling thread
// failed (or a launcher refused its shape) since the previous op.
#pragma once
#include <c10/util/Exception.h>

#include "kernels/launchers.h"

namespace tds_bind {

inline void check_launches(const char* op) {
  char buf[256];
  if (tds_take_launch_error(buf, (int)sizeof(buf))) TORCH_CHECK(false, "tdsa.", op, ": ", buf);
}

}  // namespace tds_bind
