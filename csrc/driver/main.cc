// accel-sim.out compatible command line:
//   accel-sim.out -trace ./traces/kernelslist.g -config gpgpusim.config -config trace.config [-sim_engine gpu]
#include <cstdio>
#include <string>
#include <vector>

#include "simulator.h"

int main(int argc, char** argv) {
  std::vector<std::string> args;
  for (int i = 1; i < argc; ++i) args.emplace_back(argv[i]);
  try {
    asim::Simulator sim(args);
    return sim.run();
  } catch (const std::exception& e) {
    fprintf(stderr, "\n\nGPGPU-Sim ** ERROR: %s\n", e.what());
    return 1;
  }
}
