// fvad-simulator: `simulator -i plan.json` entry point (simulator.zig:74-139).
#include "../../include/fvad.h"

int main(int argc, char **argv) { return fvad_simulator_main(argc, argv); }
