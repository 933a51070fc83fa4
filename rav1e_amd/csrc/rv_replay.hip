// rv_replay.hip -- hot-path replay driver (placeholder until the schedule
// lands; see DESIGN.md "Replay driver").
#include "rv_device.h"

struct rv_replay {
  int dummy;
};

extern "C" {
rv_replay *rv_replay_create(const rv_replay_cfg *, void *) {
  rv_set_error(RV_ENOTSUP, "rv_replay_create: not built yet");
  return nullptr;
}
void rv_replay_destroy(rv_replay *) {}
int rv_replay_set_frame(rv_replay *, int, const void *) { return RV_ENOTSUP; }
int rv_replay_frame(rv_replay *, int) { return RV_ENOTSUP; }
int rv_replay_results(rv_replay *, uint64_t *, int) { return RV_ENOTSUP; }
int rv_replay_stage_times(rv_replay *, float *, int) { return RV_ENOTSUP; }
}
