// acmmp.hpp — C++ shim over the C-ABI of libacmmp_amd.so with the member
// names of the reference's `class ACMMP` (src/ACMMP.h:58-124), for C++ callers
// such as ProcessProblem (src/acmmp_definitions.cpp:245-403). Header-only; no
// OpenCV, no HIP headers: cv::Mat / cv::Point / float4 in the reference's
// signatures become the small POD types below (INTEGRATION.md shows the
// adaptor a maintainer adds on the reference side).
//
// Errors: the reference exit()s on CUDA failures (src/ACMMP.cpp:67-75); this
// shim throws acmmp::Error carrying acmmp_last_error().
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "acmmp.h"

namespace acmmp {

struct Float4 {  // CUDA float4 of the reference's plane hypotheses
    float x, y, z, w;
};
struct Point {  // cv::Point
    int x, y;
};
struct Triangle {  // struct Triangle (src/acmmp_definitions.h:65-68)
    Point pt1, pt2, pt3;
};
struct Image {  // cv::Mat_<float>, row-major
    int rows = 0, cols = 0;
    std::vector<float> data;
    float &operator()(int r, int c) { return data[(size_t)r * cols + c]; }
    float operator()(int r, int c) const { return data[(size_t)r * cols + c]; }
};
using Problem = acmmp_problem;  // struct Problem (src/acmmp_definitions.h:57-63)
using Camera = acmmp_camera;    // struct Camera (src/acmmp_definitions.h:47-55)

// struct Problem with a std::vector of sources -> the fixed-size C layout
inline Problem make_problem(int ref_image_id, const std::vector<int> &src_image_ids, int max_image_size = 6400,
                            int num_downscale = 0, int cur_image_size = 6400) {
    Problem p{};
    p.ref_image_id = ref_image_id;
    for (int id : src_image_ids)
        if (p.num_src_images < ACMMP_MAX_IMAGES - 1) p.src_image_ids[p.num_src_images++] = id;
    p.max_image_size = max_image_size;
    p.num_downscale = num_downscale;
    p.cur_image_size = cur_image_size;
    return p;
}

class Error : public std::runtime_error {
   public:
    Error(const std::string &what, int status) : std::runtime_error(what), status_(status) {}
    int status() const { return status_; }

   private:
    int status_;
};

class ACMMP {
   public:
    explicit ACMMP(int device = 0) { check(acmmp_create(device, &ctx_), "acmmp_create"); }
    ~ACMMP() { acmmp_destroy(ctx_); }
    ACMMP(const ACMMP &) = delete;
    ACMMP &operator=(const ACMMP &) = delete;

    // ---- parameter setters (src/ACMMP.cpp:447-464)
    void SetGeomConsistencyParams(bool multi_geometry = false) {
        check(acmmp_set_geom_consistency_params(ctx_, multi_geometry ? 1 : 0), "SetGeomConsistencyParams");
    }
    void SetHierarchyParams() { check(acmmp_set_hierarchy_params(ctx_), "SetHierarchyParams"); }
    void SetPlanarPriorParams() { check(acmmp_set_planar_prior_params(ctx_), "SetPlanarPriorParams"); }
    acmmp_params params() const {
        acmmp_params p;
        check(acmmp_get_params(ctx_, &p), "acmmp_get_params");
        return p;
    }
    void set_params(const acmmp_params &p) { check(acmmp_set_params(ctx_, &p), "acmmp_set_params"); }

    // ---- input (src/ACMMP.cpp:525-809)
    void InputInitialization(const std::string &dense_folder, const std::string &output_folder,
                             const std::vector<Problem> &problems, int idx) {
        check(acmmp_input_initialization(ctx_, dense_folder.c_str(), output_folder.c_str(), problems.data(),
                                         (int)problems.size(), idx),
              "InputInitialization");
    }
    void CudaSpaceInitialization(const std::string &output_folder, const Problem &problem) {
        check(acmmp_space_initialization(ctx_, output_folder.c_str(), &problem), "CudaSpaceInitialization");
    }
    // seeded plane priors (src/ACMMP.cpp:476-523); one Float4 per ref pixel
    void SetPlanarPrior(const std::vector<Float4> &prior) {
        check(acmmp_set_seed_prior(ctx_, &prior[0].x), "SetPlanarPrior");
    }

    // ---- run (src/ACMMP.cu:1378-1456)
    void RunPatchMatch() {
        check(acmmp_run_patchmatch(ctx_), "RunPatchMatch");
        planes_.clear();
        costs_.clear();
    }

    // ---- results (src/ACMMP.cpp:833-866). Bulk-fetched once per run.
    int GetReferenceImageWidth() const { return size().first; }
    int GetReferenceImageHeight() const { return size().second; }
    Image GetReferenceImage() const {
        Image im;
        im.cols = size().first;
        im.rows = size().second;
        im.data.resize((size_t)im.rows * im.cols);
        check(acmmp_get_reference_image(ctx_, im.data.data(), im.data.size()), "GetReferenceImage");
        return im;
    }
    Float4 GetPlaneHypothesis(int index) {
        fetch();
        return planes_[(size_t)index];
    }
    float GetCost(int index) {
        fetch();
        return costs_[(size_t)index];
    }
    const std::vector<Float4> &GetPlaneHypotheses() {
        fetch();
        return planes_;
    }
    const std::vector<float> &GetCosts() {
        fetch();
        return costs_;
    }
    Camera GetCamera(int index) const {
        Camera c;
        check(acmmp_get_camera(ctx_, index, &c), "GetCamera");
        return c;
    }
    float GetMinDepth() const { return params().depth_min; }
    float GetMaxDepth() const { return params().depth_max; }

    // ---- planar prior (src/ACMMP.cpp:811-831, 868-958)
    void GetSupportPoints(std::vector<Point> &support2DPoints) {
        const int cap = (GetReferenceImageWidth() / 5 + 1) * (GetReferenceImageHeight() / 5 + 1);
        std::vector<int32_t> xy((size_t)cap * 2);
        int n = 0;
        check(acmmp_get_support_points(ctx_, xy.data(), cap, &n), "GetSupportPoints");
        support2DPoints.resize((size_t)n);
        for (int i = 0; i < n; ++i) support2DPoints[(size_t)i] = {xy[2 * i], xy[2 * i + 1]};
    }
    std::vector<Triangle> DelaunayTriangulation(int width, int height, const std::vector<Point> &points) const {
        std::vector<int32_t> xy(points.size() * 2);
        for (size_t i = 0; i < points.size(); ++i) {
            xy[2 * i] = points[i].x;
            xy[2 * i + 1] = points[i].y;
        }
        const int cap = 2 * (int)points.size() + 16;
        std::vector<int32_t> t((size_t)cap * 6);
        int n = 0;
        check(acmmp_delaunay_triangulation(width, height, xy.data(), (int)points.size(), t.data(), cap, &n),
              "DelaunayTriangulation");
        std::vector<Triangle> out((size_t)n);
        for (int i = 0; i < n; ++i)
            out[(size_t)i] = {{t[6 * i], t[6 * i + 1]}, {t[6 * i + 2], t[6 * i + 3]}, {t[6 * i + 4], t[6 * i + 5]}};
        return out;
    }
    Float4 GetPriorPlaneParams(const Triangle &tri, const Image &depths) const {
        const Camera c = GetCamera(0);
        const int32_t t[6] = {tri.pt1.x, tri.pt1.y, tri.pt2.x, tri.pt2.y, tri.pt3.x, tri.pt3.y};
        const float d[3] = {depths(tri.pt1.y, tri.pt1.x), depths(tri.pt2.y, tri.pt2.x), depths(tri.pt3.y, tri.pt3.x)};
        Float4 n4;
        check(acmmp_prior_plane_params(&c, t, d, &n4.x), "GetPriorPlaneParams");
        return n4;
    }
    float GetDepthFromPlaneParam(const Float4 &plane, int x, int y) const {
        const Camera c = GetCamera(0);
        return acmmp_depth_from_plane_param(&c, &plane.x, x, y);
    }
    // labels: 0 = none, k = plane k-1 (the reference's Mat_<float> mask)
    void CudaPlanarPriorInitialization(const std::vector<Float4> &PlaneParams, const std::vector<uint32_t> &masks) {
        check(acmmp_set_planar_prior(ctx_, PlaneParams.empty() ? nullptr : &PlaneParams[0].x,
                                     (int)PlaneParams.size(), masks.data()),
              "CudaPlanarPriorInitialization");
    }
    // The whole planar block of ProcessProblem on the device: support points,
    // Delaunay, raster, plane fit, range check, prior upload, SetPlanarPriorParams.
    std::pair<int, int> PreparePlanarPrior() {
        int np = 0, nt = 0;
        check(acmmp_prepare_planar_prior(ctx_, &np, &nt), "acmmp_prepare_planar_prior");
        return {np, nt};
    }

    acmmp_ctx *handle() const { return ctx_; }

   private:
    std::pair<int, int> size() const {
        int w = 0, h = 0;
        check(acmmp_get_reference_size(ctx_, &w, &h), "acmmp_get_reference_size");
        return {w, h};
    }
    void fetch() {
        if (!planes_.empty()) return;
        const size_t P = (size_t)GetReferenceImageWidth() * GetReferenceImageHeight();
        planes_.resize(P);
        costs_.resize(P);
        check(acmmp_get_plane_hypotheses(ctx_, &planes_[0].x, P), "GetPlaneHypothesis");
        check(acmmp_get_costs(ctx_, costs_.data(), P), "GetCost");
    }
    void check(int rc, const char *what) const {
        if (rc != ACMMP_OK) throw Error(std::string(what) + ": " + acmmp_last_error(ctx_), rc);
    }

    acmmp_ctx *ctx_ = nullptr;
    std::vector<Float4> planes_;
    std::vector<float> costs_;
};

}  // namespace acmmp
