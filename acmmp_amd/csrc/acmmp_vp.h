// acmmp_vp.h — the view-parallel multi-GPU driver of acmmp_main
// (acmmp_vp.cpp; `acmmp_main <dense> --view_parallel`).
#pragma once

#include <string>

struct VpOptions {
    std::string dense;                // dense folder (images/, cams/, pair.txt)
    std::string output_dir = "/ACMMP";
    int device = -1;                  // HIP device; -1 = LOCAL_RANK
    int iterations = 0;               // > 0 overrides max_iterations of every run
    unsigned seed = 1234;             // RNG key of view v: seed + ref id, pass index
    int geom_iterations = 2;          // geometric passes per scale (src/main_ACMMP.cpp:109)
    int concurrent_views = 2;         // engines (HIP streams) per GPU
    bool exchange_rccl = true;        // RCCL all-gather, else TCP through the rendezvous
    bool exchange_auto = true;        // no --exchange: RCCL at world > 1, a device copy at world 1
                                      // (skips the communicator's ~2.4 s initialisation)
    bool split_tail = true;           // the V mod world cheapest views in row bands over all ranks
    bool write_outputs = true;        // .dmb maps of every pass
    bool verbose = true;
};

// One rank of the view-parallel run (RANK / WORLD_SIZE / LOCAL_RANK /
// MASTER_ADDR / MASTER_PORT from the environment). 0 on success.
int run_view_parallel(const VpOptions &opt);
