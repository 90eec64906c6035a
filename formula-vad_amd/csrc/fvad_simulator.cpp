// placeholder, replaced by the plan.json simulator
#include <cstdio>
#include "../../include/fvad.h"
extern "C" int fvad_simulator_main(int, char **) {
  std::fprintf(stderr, "simulator: not implemented yet\n");
  return 1;
}
