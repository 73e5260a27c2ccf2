// acmmp_main — command-line pass driver with the options of the reference's
// main_ACMMP (src/main_ACMMP.cpp:9-176): multi-scale loop, photometric +
// planar-prior pass, two geometric-consistency passes per scale, JBU and the
// hierarchy pass on finer scales. Views are processed in order within a pass
// (the reference's Gauss-Seidel schedule). No GUI calls.
//
// After the passes it fuses the maps like main_ACMMP (:178-199) with the
// library's ports (acmmp_fusion.cpp): RunFusion into <out>/ACMMP_model.ply, or
// with -p --multi_fusion [DIR] / --force_fusion RunPriorAwareFusion against
// the reconstruction in <dense>DIR (default /ACMMP) into
// <out>/ACMMP_prior_model.ply.
#include <sys/stat.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "../../include/acmmp.h"
#include "acmmp_vp.h"

namespace {

void usage() {
    std::printf(
        "usage: acmmp_main <dense_folder> [options]\n"
        "  --output_dir NAME        output working directory name (default /ACMMP)\n"
        "  -p, --prior              seed the first pass from <dense>priors/{depths,normals}/NNNNNNNN.png\n"
        "  --device N               HIP device (default 0)\n"
        "  --iterations N           PatchMatch iterations per run (default: the reference's 2)\n"
        "  --seed N                 base RNG seed (default 1234)\n"
        "  --no_triangulation       do not write triangulation.png\n"
        "  --quiet                  no progress output\n"
        "  -f, --fuse_thresh X      average inverse score threshold for fusion (0.3)\n"
        "  --num_consistent_thresh N  consistent views needed to fuse a point (1)\n"
        "  --mask_dir DIR           boolean masks (0, 255) under <dense>/DIR\n"
        "  --image_override DIR     texture images for fusion (default /images)\n"
        "  --no_fusion              stop after the depth/normal/cost maps\n"
        "  --multi_fusion [DIR]     with -p: prior-aware fusion against <dense>DIR (default /ACMMP)\n"
        "  --force_fusion           prior-aware fusion even without -p\n"
        "  --single_match_penalty N extra consistent views required of one-sided support (0)\n"
        "  --order sequential|jacobi  pass order: the reference's (default; a geometric pass reads the maps\n"
        "                           of the views before it in the same pass) or Jacobi (= --view_parallel)\n"
        "  --view_parallel          multi-GPU: one process per GPU (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/\n"
        "                           MASTER_PORT from the environment, e.g. torchrun --no-python), views\n"
        "                           sharded per pass, depth maps all-gathered (Jacobi order); rank 0 fuses\n"
        "  --exchange rccl|tcp      view-parallel all-gather: RCCL or TCP via the rendezvous (default:\n"
        "                           RCCL at world > 1, a device copy at world 1)\n"
        "  --concurrent_views N     engines (HIP streams) per GPU (2): views in flight in the view-parallel\n"
        "                           driver, and in the sequential order's passes whose views are\n"
        "                           independent (all but multi-geometry; 1 = one at a time)\n"
        "  --no_split_tail          view-parallel: compute the V mod world tail views whole instead of\n"
        "                           in row bands over all ranks\n");
}

int die(const char *what) {
    std::fprintf(stderr, "acmmp_main: %s: %s\n", what, acmmp_pipeline_last_error());
    return 1;
}

}  // namespace

int main(int argc, char **argv) {
    std::string dense_folder, output_dir = "/ACMMP", mask_dir = " ", image_dir = "/images", fusion_dir = "/ACMMP";
    bool prior = false, quiet = false, triangulation = true, renamed_outdir = false, fusion = true;
    bool multi_fusion = false, force_fusion = false;
    float consistency_scalar = 0.3f;
    int num_consistent_thresh = 1, single_match_penalty = 0;
    int device = 0, iterations = 0, concurrent_views = 2;
    bool device_set = false, view_parallel = false, exchange_rccl = true, exchange_auto = true, split_tail = true;
    unsigned seed = 1234;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto value = [&](void) -> std::string {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "acmmp_main: %s needs a value\n", a.c_str());
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "-h" || a == "--help") {
            usage();
            return 1;  // as the reference (src/main_ACMMP.cpp:58-61)
        } else if (a == "-p" || a == "--prior") {
            prior = true;
        } else if (a == "--output_dir") {
            output_dir = value();
            renamed_outdir = true;
        } else if (a == "--device") {
            device = std::atoi(value().c_str());
            device_set = true;
        } else if (a == "--view_parallel") {
            view_parallel = true;
        } else if (a == "--order" || a.rfind("--order=", 0) == 0) {
            // one GPU offers both pass orders; jacobi = the
            // view-parallel driver at world 1 (every view of a pass reads the
            // previous pass's maps), sequential = the reference's order
            const std::string o = a == "--order" ? value() : a.substr(8);
            if (o != "sequential" && o != "jacobi") {
                std::fprintf(stderr, "acmmp_main: --order sequential|jacobi\n");
                return 2;
            }
            view_parallel = o == "jacobi";
        } else if (a == "--exchange") {
            const std::string e = value();
            if (e != "rccl" && e != "tcp") {
                std::fprintf(stderr, "acmmp_main: --exchange rccl|tcp\n");
                return 2;
            }
            exchange_rccl = e == "rccl";
            exchange_auto = false;
        } else if (a == "--no_split_tail") {
            split_tail = false;
        } else if (a == "--concurrent_views") {
            concurrent_views = std::atoi(value().c_str());
        } else if (a == "--iterations") {
            iterations = std::atoi(value().c_str());
        } else if (a == "--seed") {
            seed = (unsigned)std::strtoul(value().c_str(), nullptr, 10);
        } else if (a == "--no_triangulation") {
            triangulation = false;
        } else if (a == "--quiet") {
            quiet = true;
        } else if (a == "-f" || a == "--fuse_thresh") {
            consistency_scalar = (float)std::atof(value().c_str());
        } else if (a == "--num_consistent_thresh") {
            num_consistent_thresh = std::atoi(value().c_str());
        } else if (a == "--mask_dir") {
            mask_dir = value();
        } else if (a == "--image_override") {
            image_dir = value();
        } else if (a == "--single_match_penalty") {
            single_match_penalty = std::atoi(value().c_str());
        } else if (a == "--no_fusion") {
            fusion = false;
        } else if (a == "--multi_fusion") {
            multi_fusion = true;
            if (i + 1 < argc && argv[i + 1][0] != '-') fusion_dir = argv[++i];
        } else if (a == "--force_fusion") {
            force_fusion = true;
        } else if (!a.empty() && a[0] != '-' && dense_folder.empty()) {
            dense_folder = a;
        } else {
            std::fprintf(stderr, "acmmp_main: unknown option %s\n", a.c_str());
            usage();
            return 2;
        }
    }
    if (dense_folder.empty()) {
        usage();
        return 2;
    }

    std::vector<acmmp_problem> problems(4096);
    int num_images = 0;
    if (acmmp_generate_sample_list(dense_folder.c_str(), problems.data(), (int)problems.size(), &num_images))
        return die("GenerateSampleList");
    problems.resize((size_t)num_images);
    if (!quiet) std::printf("There are %d problems needed to be processed!\n", num_images);
    int max_num_downscale = -1;
    if (acmmp_compute_multiscale_settings(dense_folder.c_str(), problems.data(), num_images, &max_num_downscale))
        return die("ComputeMultiScaleSettings");
    // pSampler (src/main_ACMMP.cpp:72-90): priors must exist; default output
    // folder name changes unless --output_dir was given
    if (prior && !acmmp_priors_available(dense_folder.c_str(), num_images)) {
        std::printf("Initialisation from a prior was requested, but no suitable priors were found.\n");
        return -1;
    }
    if (prior && !renamed_outdir) output_dir = "/ACMMP_PRIOR";
    const std::string output_folder = dense_folder + output_dir;
    ::mkdir(output_folder.c_str(), 0777);

    acmmp_pass_options opt;
    std::memset(&opt, 0, sizeof(opt));
    opt.device = device;
    opt.max_iterations = iterations;
    opt.write_triangulation = triangulation ? 1 : 0;
    opt.verbose = quiet ? 0 : 1;
    unsigned pass = 0;
    std::string pass_error;  // the first failing view's message (set by for_views)
    // fn(0..num_images-1), `lanes` views at a time; false (and pass_error =
    // the lowest failing view's message, what the one-at-a-time loop reports)
    // if any fails
    auto for_views = [&](int lanes, auto fn) -> bool {
        lanes = std::max(1, std::min(lanes, num_images));
        std::vector<int> rc((size_t)num_images, 0);
        std::vector<std::string> msg((size_t)num_images);
        std::atomic<int> next{0};
        std::atomic<bool> failed{false};
        auto worker = [&] {
            for (int i; !failed.load() && (i = next.fetch_add(1)) < num_images;) {
                rc[(size_t)i] = fn(i);
                if (rc[(size_t)i]) {
                    msg[(size_t)i] = acmmp_pipeline_last_error();
                    failed = true;
                }
            }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < lanes; ++t) pool.emplace_back(worker);
        worker();
        for (auto &t : pool) t.join();
        for (int i = 0; i < num_images; ++i)
            if (rc[(size_t)i]) {
                pass_error = msg[(size_t)i];
                return false;
            }
        return true;
    };
    auto run_pass = [&](bool geom, bool planar, bool hier, bool multi, bool seeded = false) -> bool {
        opt.seeded = seeded;
        opt.geom_consistency = geom;
        opt.planar_prior = planar;
        opt.hierarchy = hier;
        opt.multi_geometry = multi;
        opt.seed_hi = pass++;
        // A view of a pass reads its images, its own maps of earlier passes
        // (and its own prior), and in a geometric pass its sources' depth
        // maps: depths.dmb in the first geometric pass, depths_geom.dmb in
        // the multi-geometry ones (src/ACMMP.cpp:608-635, 707-742); it writes
        // only its own folder. Only a multi-geometry pass reads files written
        // in the same pass (its earlier views' depths_geom.dmb: the
        // reference's order, src/main_ACMMP.cpp:159-172), so it runs one view
        // at a time; in every other pass the views are independent and
        // `concurrent_views` of them run at once, each with its own engine and
        // HIP stream (one view's host I/O and prior construction overlap
        // another's kernels), with the outputs of the one-at-a-time loop.
        const int lanes = (geom && multi) ? 1 : concurrent_views;
        return for_views(lanes, [&](int i) {
            acmmp_pass_options o = opt;
            o.seed_lo = seed + (unsigned)problems[(size_t)i].ref_image_id;
            return acmmp_process_problem(dense_folder.c_str(), output_folder.c_str(), problems.data(), num_images, i,
                                         &o);
        });
    };
    auto die_pass = [&](const char *what) {
        std::fprintf(stderr, "acmmp_main: %s: %s\n", what, pass_error.c_str());
        return 1;
    };

    const int geom_iterations = 2;
    if (view_parallel) {
        if (prior) {
            std::fprintf(stderr, "acmmp_main: -p is not supported with --view_parallel\n");
            return 2;
        }
        VpOptions vo;
        vo.dense = dense_folder;
        vo.output_dir = output_dir;
        vo.device = device_set ? device : -1;
        vo.iterations = iterations;
        vo.seed = seed;
        vo.geom_iterations = geom_iterations;
        vo.concurrent_views = concurrent_views;
        vo.exchange_rccl = exchange_rccl;
        vo.exchange_auto = exchange_auto;
        vo.split_tail = split_tail;
        vo.verbose = !quiet;
        const int rc = run_view_parallel(vo);
        if (rc) return rc;
        const char *r = std::getenv("RANK");
        if (r && std::atoi(r) != 0) return 0;  // rank 0 fuses
        max_num_downscale = -1;                 // the passes are done
    }
    int flag = 0;
    while (max_num_downscale >= 0) {  // src/main_ACMMP.cpp:96-176
        if (!quiet) std::printf("Scale: %d\n", max_num_downscale);
        for (auto &p : problems) {
            if (p.num_downscale >= 0) {
                p.cur_image_size = (int)(p.max_image_size / std::pow(2, p.num_downscale));
                p.num_downscale--;
            }
        }
        if (flag == 0) {
            flag = 1;
            if (!run_pass(false, true, false, false, prior)) return die_pass("ProcessProblem");
        } else {
            if (!quiet) std::printf("Starting JBU\n");
            // each view upsamples its own coarse map into its own folder: independent
            if (!for_views(concurrent_views, [&](int i) {
                    const acmmp_problem &p = problems[(size_t)i];
                    return acmmp_joint_bilateral_upsampling(dense_folder.c_str(), output_folder.c_str(), &p,
                                                            p.cur_image_size, device);
                }))
                return die_pass("JointBilateralUpsampling");
            if (!run_pass(false, true, true, false)) return die_pass("ProcessProblem");
        }
        for (int g = 0; g < geom_iterations; ++g)
            if (!run_pass(true, false, false, g > 0)) return die_pass("ProcessProblem");
        max_num_downscale--;
    }
    if (!fusion) return 0;
    int npts = 0;
    if ((prior && multi_fusion) || force_fusion) {
        const std::string fusion_folder = dense_folder + fusion_dir;
        if (acmmp_run_prior_aware_fusion(dense_folder.c_str(), output_folder.c_str(), fusion_folder.c_str(),
                                         problems.data(), num_images, 1, consistency_scalar, num_consistent_thresh,
                                         single_match_penalty, &npts)) {
            std::fprintf(stderr, "acmmp_main: RunPriorAwareFusion: %s\n", acmmp_fusion_last_error());
            return 1;
        }
        if (!quiet) std::printf("Fused %d points into %s/ACMMP_prior_model.ply\n", npts, output_folder.c_str());
        return 0;
    }
    if (acmmp_run_fusion(dense_folder.c_str(), output_folder.c_str(), problems.data(), num_images, 1,
                         consistency_scalar, num_consistent_thresh, image_dir.c_str(), mask_dir.c_str(), 1, &npts)) {
        std::fprintf(stderr, "acmmp_main: RunFusion: %s\n", acmmp_fusion_last_error());
        return 1;
    }
    if (!quiet) std::printf("Fused %d points into %s/ACMMP_model.ply\n", npts, output_folder.c_str());
    return 0;
}
