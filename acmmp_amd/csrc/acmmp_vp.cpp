// acmmp_vp.cpp — view-parallel multi-GPU pass driver in C++,
// `acmmp_main <dense> --view_parallel`: one process per GPU, the views of
// every pass sharded over the ranks, depth maps exchanged with ONE RCCL
// all-gather per pass. The same schedule as the Python driver
// (acmmp_amd/distributed.py), so the .dmb outputs are bit-identical to it:
//
//   * sharding: LPT on W*H*(N-1) of the full-size reference image;
//   * per scale (src/main_ACMMP.cpp:96-176): the images every owned view
//     needs are decoded once (acmmp_load_view) and kept in HBM; the first
//     scale runs the photometric + planar-prior pass, finer scales JBU +
//     the hierarchy pass; then two geometric passes;
//   * per view: the engine borrows the resident images
//     (acmmp_set_images_device), the gathered depth maps and the view's
//     previous state (acmmp_set_depth_maps_device /
//     acmmp_set_plane_hypotheses_device) and exports its results
//     device-to-device (acmmp_export_results); two engines per GPU, each
//     on its own HIP stream, take views off a shared queue;
//   * tail split: the V mod world cheapest views run on ALL ranks as row
//     bands (acmmp_run_patchmatch_band, 23-row halos all-gathered after
//     every half-sweep, bands all-gathered afterwards; bit-exact), each with
//     an owner rank that decodes, gathers and writes it (--no_split_tail
//     turns it off);
//   * exchange: the depth maps of a pass go through a padded
//     [world * slots, Hmax, Wmax] all-gather (ncclAllGather over xGMI, RCCL
//     has no all-gatherv). Jacobi order: every view of a pass reads the
//     previous pass's maps (the reference's second geometric pass is
//     Gauss-Seidel, src/main_ACMMP.cpp:159-172; acmmp_main without
//     --view_parallel keeps that order).
//
// Rendezvous: RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR from the
// environment (torchrun --no-python sets them); the ranks meet on TCP port
// ACMMP_RDZV_PORT (default MASTER_PORT + 1, torchrun's own store holds
// MASTER_PORT), where rank 0 hands out the ncclUniqueId. `--exchange tcp`
// all-gathers through that socket instead (host staging: several ranks on
// one GPU, where RCCL refuses duplicate devices — the 1-GPU parity tests).
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <unistd.h>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cerrno>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/acmmp.h"
#include "acmmp_vp.h"

namespace {

struct Fail : std::runtime_error {
    using std::runtime_error::runtime_error;
};

[[noreturn]] void fail(const std::string &what) { throw Fail(what); }

void hip_check(hipError_t e, const char *what) {
    if (e != hipSuccess) fail(std::string(what) + ": " + hipGetErrorString(e));
}

void acmmp_check(int rc, const char *what, const acmmp_ctx *ctx = nullptr) {
    if (rc != ACMMP_OK)
        fail(std::string(what) + " failed (status " + std::to_string(rc) + ")" +
             (ctx ? std::string(": ") + acmmp_last_error(ctx) : std::string()));
}

// ------------------------------------------------------------ rendezvous
// Rank 0 accepts world - 1 connections; each client announces its rank. The
// sockets stay open for the id broadcast, barriers and the TCP exchange.
void send_all(int fd, const void *p, size_t n) {
    const char *c = static_cast<const char *>(p);
    while (n) {
        const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
        if (k <= 0) fail("rendezvous send failed");
        c += k;
        n -= (size_t)k;
    }
}

void recv_all(int fd, void *p, size_t n) {
    char *c = static_cast<char *>(p);
    while (n) {
        const ssize_t k = ::recv(fd, c, n, 0);
        if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK))
            fail("exchange: no data from a peer within ACMMP_EXCHANGE_TIMEOUT (a rank failed or hangs)");
        if (k <= 0) fail("rendezvous recv failed (peer gone)");
        c += k;
        n -= (size_t)k;
    }
}

// Seconds a rank waits for its peers in one exchange step (a pass's
// slowest rank included) before it gives up: ACMMP_EXCHANGE_TIMEOUT, 1800.
int exchange_timeout_s() {
    const char *to = std::getenv("ACMMP_EXCHANGE_TIMEOUT");
    const int s = to && *to ? std::atoi(to) : 1800;
    return s > 0 ? s : 1800;
}

void set_socket_timeout(int fd, int seconds) {
    timeval tv{};
    tv.tv_sec = seconds;
    ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
}

class Group {
  public:
    int rank = 0, world = 1;

    Group(int rank_, int world_, const std::string &addr, int port) : rank(rank_), world(world_) {
        if (world == 1) return;
        if (rank == 0) {
            const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
            const int one = 1;
            ::setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
            sockaddr_in a{};
            a.sin_family = AF_INET;
            a.sin_port = htons((uint16_t)port);
            a.sin_addr.s_addr = htonl(INADDR_ANY);
            if (::bind(ls, (sockaddr *)&a, sizeof a) || ::listen(ls, world))
                fail("rendezvous: cannot listen on port " + std::to_string(port));
            peers_.assign(world, -1);
            const char *to = std::getenv("ACMMP_RDZV_TIMEOUT");  // seconds for every rank to arrive
            const int timeout_ms = 1000 * (to && *to ? std::atoi(to) : 600);
            for (int k = 1; k < world; ++k) {
                pollfd pf{ls, POLLIN, 0};
                if (::poll(&pf, 1, timeout_ms) != 1) {
                    ::close(ls);
                    fail("rendezvous: " + std::to_string(world - k) + " rank(s) did not connect to port " +
                         std::to_string(port) + " in time");
                }
                const int fd = ::accept(ls, nullptr, nullptr);
                if (fd < 0) fail("rendezvous accept failed");
                ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
                set_socket_timeout(fd, std::max(1, timeout_ms / 1000));  // the announcement
                int32_t r = -1;
                recv_all(fd, &r, sizeof r);
                if (r <= 0 || r >= world || peers_[r] >= 0) fail("rendezvous: bad rank announcement");
                peers_[r] = fd;
            }
            ::close(ls);
            for (int k = 1; k < world; ++k) set_socket_timeout(peers_[k], exchange_timeout_s());
        } else {
            addrinfo hints{}, *res = nullptr;
            hints.ai_family = AF_INET;
            hints.ai_socktype = SOCK_STREAM;
            if (::getaddrinfo(addr.c_str(), std::to_string(port).c_str(), &hints, &res) || !res)
                fail("rendezvous: cannot resolve " + addr);
            int fd = -1;
            for (int attempt = 0; attempt < 600 && fd < 0; ++attempt) {  // rank 0 may start later: retry 60 s
                fd = ::socket(AF_INET, SOCK_STREAM, 0);
                if (::connect(fd, res->ai_addr, res->ai_addrlen)) {
                    ::close(fd);
                    fd = -1;
                    ::usleep(100000);
                }
            }
            ::freeaddrinfo(res);
            if (fd < 0) fail("rendezvous: cannot connect to " + addr + ":" + std::to_string(port));
            const int one = 1;
            ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
            set_socket_timeout(fd, exchange_timeout_s());
            const int32_t r = rank;
            send_all(fd, &r, sizeof r);
            root_ = fd;
        }
    }

    ~Group() {
        for (int fd : peers_)
            if (fd >= 0) ::close(fd);
        if (root_ >= 0) ::close(root_);
    }

    // rank 0's bytes to every rank
    void broadcast(void *p, size_t n) {
        if (world == 1) return;
        if (rank == 0)
            for (int k = 1; k < world; ++k) send_all(peers_[k], p, n);
        else
            recv_all(root_, p, n);
    }

    // every rank's n bytes, concatenated in rank order, to every rank
    void allgather(const void *mine, void *all, size_t n) {
        char *out = static_cast<char *>(all);
        std::memcpy(out + (size_t)rank * n, mine, n);
        if (world == 1) return;
        if (rank == 0) {
            for (int k = 1; k < world; ++k) recv_all(peers_[k], out + (size_t)k * n, n);
            for (int k = 1; k < world; ++k) send_all(peers_[k], out, (size_t)world * n);
        } else {
            send_all(root_, mine, n);
            recv_all(root_, out, (size_t)world * n);
        }
    }

    void barrier() {
        char b = 0;
        std::vector<char> all((size_t)world);
        allgather(&b, all.data(), 1);
    }

  private:
    std::vector<int> peers_;
    int root_ = -1;
};

// ------------------------------------------------------------ exchange
class Exchange {
  public:
    Exchange(Group &g, bool rccl, int device) : g_(g), rccl_(rccl) {
        const auto t0 = std::chrono::steady_clock::now();
        hip_check(hipSetDevice(device), "hipSetDevice");
        hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
        if (rccl_) {
            ncclUniqueId id;
            if (g.rank == 0 && ncclGetUniqueId(&id) != ncclSuccess) fail("ncclGetUniqueId failed");
            g.broadcast(&id, sizeof id);
            const ncclResult_t r = ncclCommInitRank(&comm_, g.world, id, g.rank);
            if (r != ncclSuccess) fail(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        }
        if (std::getenv("ACMMP_HOST_TIMING"))
            std::fprintf(stderr, "[rank %d] exchange init (%s)=%.2fs\n", g.rank, rccl_ ? "rccl" : "local/tcp",
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    ~Exchange() {
        if (comm_) ncclCommDestroy(comm_);
        if (stream_) (void)hipStreamDestroy(stream_);
    }

    // d_recv[world * count] = concatenation of every rank's d_send[count]
    void allgather(const float *d_send, float *d_recv, size_t count) {
        if (rccl_) {  // world 1 included: the same RCCL call as at 8 GPUs
            const ncclResult_t r = ncclAllGather(d_send, d_recv, count, ncclFloat32, comm_, stream_);
            if (r != ncclSuccess) fail(std::string("ncclAllGather: ") + ncclGetErrorString(r));
            wait_rccl();
            return;
        } else if (g_.world == 1) {
            hip_check(hipMemcpyAsync(d_recv, d_send, count * sizeof(float), hipMemcpyDeviceToDevice, stream_),
                      "hipMemcpyAsync");
        } else {
            std::vector<float> mine(count), all(count * (size_t)g_.world);
            hip_check(hipMemcpy(mine.data(), d_send, count * sizeof(float), hipMemcpyDeviceToHost), "hipMemcpy");
            g_.allgather(mine.data(), all.data(), count * sizeof(float));
            hip_check(hipMemcpy(d_recv, all.data(), all.size() * sizeof(float), hipMemcpyHostToDevice), "hipMemcpy");
        }
        // the engines' streams do not wait on this one
        hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    }

  private:
    // the all-gather has finished, or the communicator reported an error /
    // the peers did not arrive within ACMMP_EXCHANGE_TIMEOUT: then abort it
    // (the peers' collectives fail too) and exit non-zero instead of blocking
    void wait_rccl() {
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(exchange_timeout_s());
        for (;;) {
            const hipError_t q = hipStreamQuery(stream_);
            if (q == hipSuccess) return;
            if (q != hipErrorNotReady) hip_check(q, "ncclAllGather stream");
            ncclResult_t async = ncclSuccess;
            if (ncclCommGetAsyncError(comm_, &async) != ncclSuccess || async != ncclSuccess) {
                abort_comm();
                fail(std::string("ncclAllGather: ") + ncclGetErrorString(async));
            }
            if (std::chrono::steady_clock::now() > deadline) {
                abort_comm();
                fail("ncclAllGather: peers did not arrive within ACMMP_EXCHANGE_TIMEOUT");
            }
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }
    void abort_comm() {
        (void)ncclCommAbort(comm_);
        comm_ = nullptr;
    }

    Group &g_;
    bool rccl_;
    ncclComm_t comm_ = nullptr;
    hipStream_t stream_ = nullptr;
};

// ------------------------------------------------------------ buffers
struct DevBuf {
    float *p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    explicit DevBuf(size_t count) : n(count) {
        if (count) hip_check(hipMalloc((void **)&p, count * sizeof(float)), "hipMalloc");
    }
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    DevBuf(DevBuf &&o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    DevBuf &operator=(DevBuf &&o) noexcept {
        std::swap(p, o.p);
        std::swap(n, o.n);
        return *this;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

std::string image_path(const std::string &dense, int id) {
    char name[32];
    std::snprintf(name, sizeof name, "%08d", id);
    const std::string base = dense + "/images/" + name;
    for (const char *ext : {".jpg", ".pgm", ".pfm"}) {
        struct stat st;
        if (::stat((base + ext).c_str(), &st) == 0) return base + ext;
    }
    return base + ".jpg";
}

std::string result_folder(const std::string &out, int ref_id) {
    char name[32];
    std::snprintf(name, sizeof name, "/2333_%08d", ref_id);
    return out + name;
}

struct ViewState {
    DevBuf planes, costs;  // (H, W, 4) world normal + depth, (H, W)
    int W = 0, H = 0;
    DevBuf jbu;  // upsampled depth of the hierarchy pass (device, the next scale's W x H)
};

// --------------------------------------------------------------- driver
class Driver {
  public:
    Driver(const VpOptions &o, Group &g) : o_(o), g_(g), ex_(g, o.exchange_rccl, o.device) {
        output_folder_ = o.dense + o.output_dir;
        problems_.resize(4096);
        int n = 0;
        acmmp_check(acmmp_generate_sample_list(o.dense.c_str(), problems_.data(), (int)problems_.size(), &n),
                    "GenerateSampleList");
        problems_.resize((size_t)n);
        acmmp_check(acmmp_compute_multiscale_settings(o.dense.c_str(), problems_.data(), n, &max_down_),
                    "ComputeMultiScaleSettings");
        for (int i = 0; i < n; ++i) index_of_[problems_[(size_t)i].ref_image_id] = i;
        // LPT on W*H*max(N-1, 1) of the full-size reference image
        std::vector<double> cost((size_t)n);
        for (int i = 0; i < n; ++i) {
            int w = 0, h = 0;
            acmmp_check(acmmp_image_size(image_path(o.dense, problems_[(size_t)i].ref_image_id).c_str(), &w, &h),
                        "image header");
            cost[(size_t)i] = (double)w * h * std::max(problems_[(size_t)i].num_src_images, 1);
        }
        std::vector<int> order((size_t)n);
        for (int i = 0; i < n; ++i) order[(size_t)i] = i;
        std::sort(order.begin(), order.end(), [&](int a, int b) {
            return cost[(size_t)a] != cost[(size_t)b] ? cost[(size_t)a] > cost[(size_t)b] : a < b;
        });
        // the tail (V mod world cheapest views) is split over all ranks;
        // the rest LPT; each split view's owner is the least loaded rank
        const int ntail = (o.split_tail && g.world > 1) ? n % g.world : 0;
        split_.assign(order.end() - ntail, order.end());
        std::sort(split_.begin(), split_.end());
        std::vector<double> load((size_t)g.world, 0.0);
        assignment_.assign((size_t)g.world, {});
        auto place = [&](int v) {
            int r = 0;
            for (int k = 1; k < g.world; ++k)
                if (load[(size_t)k] < load[(size_t)r]) r = k;
            assignment_[(size_t)r].push_back(v);
            load[(size_t)r] += cost[(size_t)v];
        };
        for (int v : order)
            if (!is_split(v)) place(v);
        for (int v : split_) place(v);
        for (auto &a : assignment_) std::sort(a.begin(), a.end());
        owned_ = assignment_[(size_t)g.rank];
        for (int v : owned_)
            if (!is_split(v)) mine_.push_back(v);
        for (int k = 0; k < std::max(o.concurrent_views, 1); ++k) {
            acmmp_ctx *ctx = nullptr;
            acmmp_check(acmmp_create(o.device, &ctx), "acmmp_create");
            engines_.push_back(ctx);
            hipStream_t cs = nullptr;
            hip_check(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking), "hipStreamCreate");
            copy_.push_back(cs);
        }
    }

    ~Driver() {
        for (auto &t : writers_)
            if (t.joinable()) t.join();
        for (auto *e : engines_) acmmp_destroy(e);
        for (auto cs : copy_) (void)hipStreamDestroy(cs);
        for (auto &kv : textures_) acmmp_texture_destroy(kv.second);
    }

    void run() {
        ::mkdir(output_folder_.c_str(), 0777);
        bool first = true;
        while (max_down_ >= 0) {
            for (auto &p : problems_)  // cur_image_size for this scale (src/main_ACMMP.cpp:99-106)
                if (p.num_downscale >= 0) {
                    p.cur_image_size = (int)(p.max_image_size / std::pow(2.0, p.num_downscale));
                    p.num_downscale--;
                }
            {
                Clock c(this, "load");
                shapes();
                load_views();
            }
            if (first) {
                first = false;
                run_pass(false, true, false, false);
            } else {
                {
                    Clock c(this, "jbu");
                    jbu();
                }
                run_pass(false, true, true, false);
            }
            for (int gi = 0; gi < o_.geom_iterations; ++gi) run_pass(true, false, false, gi > 0);
            max_down_--;
        }
        {
            Clock c(this, "flush_writes");
            flush_writes();
        }
        g_.barrier();
        if (std::getenv("ACMMP_HOST_TIMING")) {
            std::fprintf(stderr, "[rank %d]", g_.rank);
            for (auto &kv : phase_s_) std::fprintf(stderr, " %s=%.2fs", kv.first.c_str(), kv.second);
            std::fprintf(stderr, "\n");
        }
    }

  private:
    struct Task {
        int v;  // problem index
        bool geom, planar, hier, multi;
    };

    // wall seconds per phase (ACMMP_HOST_TIMING=1 prints them)
    struct Clock {
        Driver *d;
        const char *name;
        std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
        Clock(Driver *d_, const char *n) : d(d_), name(n) {}
        ~Clock() {
            d->phase_s_[name] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
    };

    // the .dmb writers of the previous pass have finished (they read the
    // state buffers the next pass end replaces); their first error is raised
    void flush_writes() {
        for (auto &t : writers_) t.join();
        writers_.clear();
        for (auto &e : write_errs_)
            if (!e.empty()) fail(e);
        write_errs_.clear();
    }

    // a pass's outputs written by 4 host threads while the next pass computes
    void start_writes(bool geom) {
        const int nw = (int)std::min<size_t>(4, owned_.size());
        write_errs_.assign((size_t)nw, std::string());
        for (int w = 0; w < nw; ++w)
            writers_.emplace_back([this, w, nw, geom]() {
                try {
                    hip_check(hipSetDevice(o_.device), "hipSetDevice");
                    for (size_t k = (size_t)w; k < owned_.size(); k += (size_t)nw)
                        write_outputs(owned_[k], state_.at(owned_[k]), geom);
                } catch (const std::exception &e) {
                    write_errs_[(size_t)w] = e.what();
                }
            });
    }

    // Images of this scale, decoded once per node: every rank decodes the
    // reference images of ITS views (acmmp_load_view: JPEG decode + rescale,
    // InputInitialization src/ACMMP.cpp:536-598) and the images travel in
    // ONE padded all-gather, like the depth maps (RCCL over xGMI); cameras
    // come from the headers and cam files of every image a view needs.
    void load_views() {
        for (auto &kv : textures_) acmmp_texture_destroy(kv.second);
        textures_.clear();
        images_.clear();
        cams_.clear();
        std::vector<int> need;
        std::vector<int> compute_views = mine_;
        compute_views.insert(compute_views.end(), split_.begin(), split_.end());
        for (int v : compute_views) {
            const acmmp_problem &p = problems_[(size_t)v];
            need.push_back(p.ref_image_id);
            for (int s = 0; s < p.num_src_images; ++s) need.push_back(p.src_image_ids[s]);
        }
        std::sort(need.begin(), need.end());
        need.erase(std::unique(need.begin(), need.end()), need.end());
        for (int id : need)
            if (!index_of_.count(id)) fail("source id " + std::to_string(id) + " is not a problem index");
        // work items: the cameras of every needed image, the pixels of my refs
        std::vector<acmmp_camera> cams(need.size());
        std::vector<std::vector<float>> host(owned_.size());
        std::vector<acmmp_camera> own_cams(owned_.size());
        const size_t nwork = need.size() + owned_.size();
        std::vector<std::string> errs(nwork);
        std::atomic<size_t> next{0};
        auto worker = [&]() {
            for (size_t k; (k = next++) < nwork;) {
                const bool pixels = k >= need.size();
                const int v = pixels ? owned_[k - need.size()] : -1;
                const int id = pixels ? problems_[(size_t)v].ref_image_id : need[k];
                acmmp_camera &cam = pixels ? own_cams[k - need.size()] : cams[k];
                const int size = problems_[(size_t)index_of_.at(id)].cur_image_size;
                int rc = acmmp_load_view(o_.dense.c_str(), id, size, nullptr, 0, &cam);
                if (rc != ACMMP_OK && rc != ACMMP_ERR_ARG) {
                    errs[k] = std::string("acmmp_load_view: ") + acmmp_pipeline_last_error();
                    continue;
                }
                if (!pixels) continue;
                std::vector<float> &h = host[k - need.size()];
                h.resize((size_t)cam.width * cam.height);
                rc = acmmp_load_view(o_.dense.c_str(), id, size, h.data(), h.size(), &cam);
                if (rc != ACMMP_OK) errs[k] = std::string("acmmp_load_view: ") + acmmp_pipeline_last_error();
            }
        };
        std::vector<std::thread> pool;
        const int nt = (int)std::min<size_t>((size_t)acmmp_host_threads(), nwork);
        for (int t = 0; t < nt; ++t) pool.emplace_back(worker);
        for (auto &t : pool) t.join();
        for (size_t k = 0; k < nwork; ++k)
            if (!errs[k].empty())
                fail("view " + std::to_string(k < need.size() ? need[k] : problems_[(size_t)owned_[k - need.size()]].ref_image_id) +
                     ": " + errs[k]);
        // my refs: kept contiguous for JBU, and padded into my all-gather slots
        DevBuf send((size_t)slots_ * hmax_ * wmax_);
        hip_check(hipMemset(send.p, 0, send.n * sizeof(float)), "hipMemset");
        for (size_t k = 0; k < owned_.size(); ++k) {
            const acmmp_camera &c = own_cams[k];
            const int v = owned_[k];
            if (c.height != shape_[(size_t)v].first || c.width != shape_[(size_t)v].second)
                fail("view " + std::to_string(problems_[(size_t)v].ref_image_id) + ": image size disagrees with its header");
            DevBuf d(host[k].size());
            hip_check(hipMemcpy(d.p, host[k].data(), host[k].size() * sizeof(float), hipMemcpyHostToDevice), "hipMemcpy");
            hip_check(hipMemcpy2D(send.p + k * (size_t)hmax_ * wmax_, (size_t)wmax_ * sizeof(float), d.p,
                                  (size_t)c.width * sizeof(float), (size_t)c.width * sizeof(float), (size_t)c.height,
                                  hipMemcpyDeviceToDevice),
                      "hipMemcpy2D");
            images_.emplace(problems_[(size_t)v].ref_image_id, std::move(d));
        }
        hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
        recv_img_ = DevBuf(send.n * (size_t)g_.world);
        ex_.allgather(send.p, recv_img_.p, send.n);
        // the padded footprint records, built once per image and scale from
        // the gathered image (row pitch Wmax)
        for (size_t k = 0; k < need.size(); ++k) {
            const acmmp_camera &c = cams[k];
            const float *img = gathered_in(recv_img_, index_of_.at(need[k]));
            acmmp_texture *t = nullptr;
            acmmp_check(acmmp_texture_create(o_.device, img, wmax_, c.width, c.height, &t), "acmmp_texture_create");
            textures_[need[k]] = t;
            cams_[need[k]] = c;
        }
        // a split view's JBU runs on every rank: its reference image, unpadded
        for (int v : split_) {
            const int id = problems_[(size_t)v].ref_image_id;
            if (images_.count(id)) continue;
            const acmmp_camera &c = cams_.at(id);
            DevBuf d((size_t)c.width * c.height);
            hip_check(hipMemcpy2DAsync(d.p, (size_t)c.width * sizeof(float), gathered_in(recv_img_, v),
                                       (size_t)wmax_ * sizeof(float), (size_t)c.width * sizeof(float),
                                       (size_t)c.height, hipMemcpyDeviceToDevice, copy_[0]),
                      "hipMemcpy2DAsync");
            hip_check(hipStreamSynchronize(copy_[0]), "hipStreamSynchronize");
            images_.emplace(id, std::move(d));
        }
    }

    // (h, w) of every view at this scale (acmmp_load_view's rescale rule)
    void shapes() {
        shape_.assign(problems_.size(), {0, 0});
        int hmax = 0, wmax = 0;
        for (size_t i = 0; i < problems_.size(); ++i) {
            int w = 0, h = 0;
            acmmp_check(acmmp_image_size(image_path(o_.dense, problems_[i].ref_image_id).c_str(), &w, &h),
                        "image header");
            const int m = problems_[i].cur_image_size;
            if (w > m || h > m) {
                const float f = std::min((float)m / (float)w, (float)m / (float)h);
                w = (int)std::nearbyint((float)w * f);
                h = (int)std::nearbyint((float)h * f);
            }
            shape_[i] = {h, w};
            hmax = std::max(hmax, h);
            wmax = std::max(wmax, w);
        }
        if (!split_checked_) {  // every band must hold the halo at the coarsest scale (this one)
            split_checked_ = true;
            std::vector<int> keep;
            for (int v : split_) {
                if (shape_[(size_t)v].first >= g_.world * ACMMP_BAND_HALO) {
                    keep.push_back(v);
                } else if (std::find(owned_.begin(), owned_.end(), v) != owned_.end()) {
                    mine_.push_back(v);  // its owner computes it whole
                    std::sort(mine_.begin(), mine_.end());
                }
            }
            split_ = keep;
        }
        slots_ = 1;
        for (auto &a : assignment_) slots_ = std::max(slots_, (int)a.size());
        hmax_ = hmax;
        wmax_ = wmax;
        const size_t per = (size_t)slots_ * hmax_ * wmax_;
        send_ = DevBuf(per);
        recv_ = DevBuf(per * (size_t)g_.world);
        depth_tmp_.clear();
    }

    acmmp_params view_params(const Task &t) const {
        acmmp_params p;
        acmmp_default_params(&p);
        if (t.geom) {  // SetGeomConsistencyParams (src/ACMMP.cpp:447-454)
            p.geom_consistency = 1;
            p.max_iterations = 2;
            if (t.multi) p.multi_geometry = 1;
        }
        if (t.hier) p.hierarchy = 1;
        const acmmp_problem &pr = problems_[(size_t)t.v];
        p.seed_lo = o_.seed + (unsigned)pr.ref_image_id;
        p.seed_hi = (unsigned)pass_index_;
        if (o_.iterations > 0) p.max_iterations = o_.iterations;
        return p;
    }

    // problem i's map in a padded all-gather buffer (row pitch Wmax)
    const float *gathered_in(const DevBuf &buf, int i) const {
        for (int r = 0; r < g_.world; ++r) {
            const auto &a = assignment_[(size_t)r];
            for (size_t k = 0; k < a.size(); ++k)
                if (a[k] == i) return buf.p + ((size_t)r * slots_ + k) * hmax_ * wmax_;
        }
        fail("view not assigned");
    }
    // the gathered depth map of problem i (previous pass)
    const float *gathered(int i) const { return gathered_in(recv_, i); }

    void compute(acmmp_ctx *eng, const Task &t, ViewState &out, hipStream_t cs, bool band = false) {
        const acmmp_problem &pr = problems_[(size_t)t.v];
        std::vector<int> ids = {pr.ref_image_id};
        for (int s = 0; s < pr.num_src_images; ++s) ids.push_back(pr.src_image_ids[s]);
        std::vector<acmmp_camera> cams;
        std::vector<const acmmp_texture *> tex;
        for (int id : ids) {
            cams.push_back(cams_.at(id));
            tex.push_back(textures_.at(id));
        }
        const acmmp_params p = view_params(t);
        acmmp_check(acmmp_set_params(eng, &p), "acmmp_set_params", eng);
        acmmp_check(acmmp_set_images_textures(eng, (int)ids.size(), cams.data(), tex.data(), 0),
                    "acmmp_set_images_textures", eng);
        const int W = cams[0].width, H = cams[0].height;
        ViewState &prev = state_[t.v];
        if (t.geom) {
            std::vector<const float *> deps;
            std::vector<int32_t> pitches;
            for (int id : ids) {
                deps.push_back(gathered(index_of_.at(id)));
                pitches.push_back(wmax_);
            }
            acmmp_check(acmmp_set_depth_maps_device(eng, deps.data(), pitches.data()), "acmmp_set_depth_maps_device",
                        eng);
            acmmp_check(acmmp_set_plane_hypotheses_device(eng, prev.planes.p, prev.costs.p),
                        "acmmp_set_plane_hypotheses_device", eng);
        }
        DevBuf scaled;  // alive until the run below has been synchronised
        if (t.hier) {  // scaled planes = previous scale's normals + (costs, or the JBU depth when no upsample)
            const int sh = prev.H, sw = prev.W;
            const size_t S = (size_t)sh * sw;
            const bool upsample = sw != H || sh != W;  // src/ACMMP.cpp:766, rows/cols swap included
            if (!upsample && prev.jbu.n < S) fail("hierarchy input: JBU depth smaller than the scaled planes");
            scaled = DevBuf(S * 4);
            // built on the device: the normals, then the 4th channel as a
            // strided copy (4 of every 16 bytes), as the Python driver does
            // (device-to-device hipMemcpy does not wait for the copy, and the
            // engine stream is non-blocking: copy on `cs` and wait for it)
            hip_check(hipMemcpyAsync(scaled.p, prev.planes.p, S * 4 * sizeof(float), hipMemcpyDeviceToDevice, cs),
                      "hipMemcpyAsync");
            hip_check(hipMemcpy2DAsync(scaled.p + 3, 4 * sizeof(float), upsample ? prev.costs.p : prev.jbu.p,
                                       sizeof(float), sizeof(float), S, hipMemcpyDeviceToDevice, cs),
                      "hipMemcpy2DAsync");
            hip_check(hipStreamSynchronize(cs), "hipStreamSynchronize");
            acmmp_check(acmmp_set_hierarchy_inputs_device(eng, scaled.p, sw, sh, prev.jbu.p),
                        "acmmp_set_hierarchy_inputs_device", eng);
        }
        out.W = W;
        out.H = H;
        out.planes = DevBuf((size_t)W * H * 4);
        out.costs = DevBuf((size_t)W * H);
        DevBuf depth((size_t)W * H);
        if (band) {
            run_band(eng, t, out, depth, cs);
        } else {
            acmmp_check(acmmp_run_patchmatch_async(eng), "acmmp_run_patchmatch_async", eng);
            if (t.planar) {
                acmmp_check(acmmp_synchronize(eng), "acmmp_synchronize", eng);
                int nsp = 0, ntri = 0;
                acmmp_check(acmmp_prepare_planar_prior(eng, &nsp, &ntri), "acmmp_prepare_planar_prior", eng);
                acmmp_check(acmmp_run_patchmatch_async(eng), "acmmp_run_patchmatch_async", eng);
            }
            acmmp_check(acmmp_export_results(eng, out.planes.p, out.costs.p, depth.p), "acmmp_export_results", eng);
            acmmp_check(acmmp_synchronize(eng), "acmmp_synchronize", eng);
        }
        std::lock_guard<std::mutex> lk(mu_);
        depth_tmp_[t.v] = std::move(depth);
    }

    bool is_split(int v) const { return std::find(split_.begin(), split_.end(), v) != split_.end(); }

    // rows [lo, hi) of band k of H rows over the world (sizes differ by at most 1)
    std::pair<int, int> band_rows(int H, int k) const {
        const int base = H / g_.world, extra = H % g_.world;
        const int lo = k * base + std::min(k, extra);
        return {lo, lo + base + (k < extra ? 1 : 0)};
    }

    // The halo exchange of a band run (acmmp_run_patchmatch_band's callback):
    // each rank all-gathers [rows the band above reads | rows the band below
    // reads] of the colour just written (plane float4, cost, selected views),
    // then takes its neighbours' parts. One all-gather of 2 x 23 rows per
    // rank and half-sweep (RCCL over xGMI, or the TCP exchange).
    struct BandCtx {
        Driver *d;
        hipStream_t cs;
        DevBuf send, recv;
        std::string err;
    };
    static int band_exchange(void *user, const acmmp_band_halo *h) {
        BandCtx *b = static_cast<BandCtx *>(user);
        try {
            b->d->halo_exchange(*b, *h);
            return 0;
        } catch (const std::exception &e) {
            b->err = e.what();
            return 1;
        }
    }
    void halo_exchange(BandCtx &b, const acmmp_band_halo &h) {
        const size_t Wh = (size_t)h.Wh, K = ACMMP_BAND_HALO;
        const size_t part = K * Wh * 6;  // floats: K rows of plane (4) + cost + selected views
        if (b.send.n != 2 * part) {
            b.send = DevBuf(2 * part);
            b.recv = DevBuf(2 * part * (size_t)g_.world);
        }
        // the sweep that wrote these rows ran on the engine's stream
        hip_check(hipStreamSynchronize((hipStream_t)h.stream), "hipStreamSynchronize");
        auto pack = [&](float *dst, int lo, int hi) {
            const size_t n = (size_t)(hi - lo) * Wh;
            if (!n) return;
            hip_check(hipMemcpyAsync(dst, (const float *)h.plane + (size_t)lo * Wh * 4, n * 16, hipMemcpyDeviceToDevice,
                                     b.cs), "hipMemcpyAsync");
            hip_check(hipMemcpyAsync(dst + K * Wh * 4, (const float *)h.cost + (size_t)lo * Wh, n * 4,
                                     hipMemcpyDeviceToDevice, b.cs), "hipMemcpyAsync");
            hip_check(hipMemcpyAsync(dst + K * Wh * 5, (const uint32_t *)h.sv + (size_t)lo * Wh, n * 4,
                                     hipMemcpyDeviceToDevice, b.cs), "hipMemcpyAsync");
        };
        auto unpack = [&](const float *src, int lo, int hi) {
            const size_t n = (size_t)(hi - lo) * Wh;
            if (!n) return;
            hip_check(hipMemcpyAsync((float *)h.plane + (size_t)lo * Wh * 4, src, n * 16, hipMemcpyDeviceToDevice, b.cs),
                      "hipMemcpyAsync");
            hip_check(hipMemcpyAsync((float *)h.cost + (size_t)lo * Wh, src + K * Wh * 4, n * 4,
                                     hipMemcpyDeviceToDevice, b.cs), "hipMemcpyAsync");
            hip_check(hipMemcpyAsync((uint32_t *)h.sv + (size_t)lo * Wh, src + K * Wh * 5, n * 4,
                                     hipMemcpyDeviceToDevice, b.cs), "hipMemcpyAsync");
        };
        pack(b.send.p, h.send_up_lo, h.send_up_hi);
        pack(b.send.p + part, h.send_down_lo, h.send_down_hi);
        hip_check(hipStreamSynchronize(b.cs), "hipStreamSynchronize");
        ex_.allgather(b.send.p, b.recv.p, b.send.n);
        const int r = g_.rank;
        if (r > 0) unpack(b.recv.p + (size_t)(r - 1) * 2 * part + part, h.recv_up_lo, h.recv_up_hi);
        if (r + 1 < g_.world) unpack(b.recv.p + (size_t)(r + 1) * 2 * part, h.recv_down_lo, h.recv_down_hi);
        // the engine's next sweep is enqueued after this returns
        hip_check(hipStreamSynchronize(b.cs), "hipStreamSynchronize");
    }

    // every band's rows of the exported (planes, costs) from its rank, on every rank
    void gather_bands(ViewState &out, hipStream_t cs) {
        const int W = out.W, H = out.H;
        int rmax = 0;
        for (int k = 0; k < g_.world; ++k) rmax = std::max(rmax, band_rows(H, k).second - band_rows(H, k).first);
        const size_t per = (size_t)rmax * W * 5;
        DevBuf send(per), recv(per * (size_t)g_.world);
        const auto [lo, hi] = band_rows(H, g_.rank);
        hip_check(hipMemcpyAsync(send.p, out.planes.p + (size_t)lo * W * 4, (size_t)(hi - lo) * W * 16,
                                 hipMemcpyDeviceToDevice, cs), "hipMemcpyAsync");
        hip_check(hipMemcpyAsync(send.p + (size_t)rmax * W * 4, out.costs.p + (size_t)lo * W, (size_t)(hi - lo) * W * 4,
                                 hipMemcpyDeviceToDevice, cs), "hipMemcpyAsync");
        hip_check(hipStreamSynchronize(cs), "hipStreamSynchronize");
        ex_.allgather(send.p, recv.p, per);
        for (int k = 0; k < g_.world; ++k) {
            if (k == g_.rank) continue;
            const auto [blo, bhi] = band_rows(H, k);
            const float *src = recv.p + (size_t)k * per;
            hip_check(hipMemcpyAsync(out.planes.p + (size_t)blo * W * 4, src, (size_t)(bhi - blo) * W * 16,
                                     hipMemcpyDeviceToDevice, cs), "hipMemcpyAsync");
            hip_check(hipMemcpyAsync(out.costs.p + (size_t)blo * W, src + (size_t)rmax * W * 4,
                                     (size_t)(bhi - blo) * W * 4, hipMemcpyDeviceToDevice, cs), "hipMemcpyAsync");
        }
        hip_check(hipStreamSynchronize(cs), "hipStreamSynchronize");
    }

    // One view's run split in row bands over every rank (the engine already
    // holds the view's inputs): this rank's band, the halos exchanged every
    // half-sweep, the bands gathered; with the planar prior, the prior is
    // rebuilt on every rank from the gathered first run, then the second run
    // (src/acmmp_definitions.cpp:306-379). `depth` = the planes' w channel.
    void run_band(acmmp_ctx *eng, const Task &t, ViewState &out, DevBuf &depth, hipStream_t cs) {
        const auto [lo, hi] = band_rows(out.H, g_.rank);
        BandCtx b{this, cs, {}, {}, {}};
        for (int run = 0; run < (t.planar ? 2 : 1); ++run) {
            if (run) {
                acmmp_check(acmmp_set_plane_hypotheses_device(eng, out.planes.p, out.costs.p),
                            "acmmp_set_plane_hypotheses_device", eng);
                int nsp = 0, ntri = 0;
                acmmp_check(acmmp_prepare_planar_prior(eng, &nsp, &ntri), "acmmp_prepare_planar_prior", eng);
            }
            const int rc = acmmp_run_patchmatch_band(eng, lo, hi, &Driver::band_exchange, &b);
            if (!b.err.empty()) fail("band exchange: " + b.err);
            acmmp_check(rc, "acmmp_run_patchmatch_band", eng);
            acmmp_check(acmmp_export_results(eng, out.planes.p, out.costs.p, nullptr), "acmmp_export_results", eng);
            acmmp_check(acmmp_synchronize(eng), "acmmp_synchronize", eng);
            gather_bands(out, cs);
        }
        const size_t P = (size_t)out.W * out.H;
        hip_check(hipMemcpy2DAsync(depth.p, sizeof(float), out.planes.p + 3, 4 * sizeof(float), sizeof(float), P,
                                   hipMemcpyDeviceToDevice, cs),
                  "hipMemcpy2DAsync");
        hip_check(hipStreamSynchronize(cs), "hipStreamSynchronize");
    }

    void write_outputs(int v, const ViewState &s, bool geom) {
        const std::string folder = result_folder(output_folder_, problems_[(size_t)v].ref_image_id);
        ::mkdir(folder.c_str(), 0777);
        const size_t P = (size_t)s.W * s.H;
        std::vector<float> pl(P * 4), co(P), d(P), n(P * 3);
        hip_check(hipMemcpy(pl.data(), s.planes.p, pl.size() * sizeof(float), hipMemcpyDeviceToHost), "hipMemcpy");
        hip_check(hipMemcpy(co.data(), s.costs.p, co.size() * sizeof(float), hipMemcpyDeviceToHost), "hipMemcpy");
        for (size_t k = 0; k < P; ++k) {
            d[k] = pl[4 * k + 3];
            n[3 * k + 0] = pl[4 * k + 0];
            n[3 * k + 1] = pl[4 * k + 1];
            n[3 * k + 2] = pl[4 * k + 2];
        }
        const std::string dn = folder + (geom ? "/depths_geom.dmb" : "/depths.dmb");
        if (acmmp_write_dmb(dn.c_str(), s.H, s.W, 1, d.data()) ||
            acmmp_write_dmb((folder + "/normals.dmb").c_str(), s.H, s.W, 3, n.data()) ||
            acmmp_write_dmb((folder + "/costs.dmb").c_str(), s.H, s.W, 1, co.data()))
            fail("cannot write the .dmb outputs of view " + std::to_string(problems_[(size_t)v].ref_image_id));
    }

    void run_pass(bool geom, bool planar, bool hier, bool multi) {
        std::vector<Task> tasks;
        for (int v : mine_) tasks.push_back({v, geom, planar, hier, multi});
        std::map<int, ViewState> next;
        for (int v : mine_) {  // every key exists before the worker threads look them up
            next[v];
            state_[v];
        }
        for (int v : split_) {
            next[v];
            state_[v];
        }
        // views off a shared queue, one host thread per engine
        std::atomic<size_t> q{0};
        std::vector<std::string> errs(engines_.size());
        auto worker = [&](size_t e) {
            try {
                hip_check(hipSetDevice(o_.device), "hipSetDevice");  // per thread: the output buffers go there
                for (size_t k; (k = q++) < tasks.size();) compute(engines_[e], tasks[k], next[tasks[k].v], copy_[e]);
            } catch (const std::exception &ex) {
                errs[e] = ex.what();
                q = tasks.size();
            }
        };
        {
            Clock c(this, "compute");
            std::vector<std::thread> th;
            for (size_t e = 0; e < engines_.size(); ++e) th.emplace_back(worker, e);
            for (auto &t : th) t.join();
        }
        for (auto &e : errs)
            if (!e.empty()) fail(e);
        if (!split_.empty()) {  // the tail views, every rank on a band of each
            Clock c(this, "split_compute");
            for (int v : split_) compute(engines_[0], Task{v, geom, planar, hier, multi}, next[v], copy_[0], true);
        }
        {
            Clock c(this, "flush_writes");
            flush_writes();  // the previous pass's writers still read the state replaced below
        }
        Clock c(this, "exchange");
        // state, then the padded all-gather of the depth maps; the outputs are
        // written while the next pass computes
        hip_check(hipMemset(send_.p, 0, send_.n * sizeof(float)), "hipMemset");
        for (int v : split_)  // every rank holds the split views' full state
            if (std::find(owned_.begin(), owned_.end(), v) == owned_.end()) state_[v] = std::move(next[v]);
        for (size_t k = 0; k < owned_.size(); ++k) {
            const int v = owned_[k];
            ViewState &s = next[v];
            hip_check(hipMemcpy2D(send_.p + k * (size_t)hmax_ * wmax_, (size_t)wmax_ * sizeof(float),
                                  depth_tmp_.at(v).p, (size_t)s.W * sizeof(float), (size_t)s.W * sizeof(float),
                                  (size_t)s.H, hipMemcpyDeviceToDevice),
                      "hipMemcpy2D");
            state_[v] = std::move(s);
        }
        hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
        depth_tmp_.clear();
        if (o_.write_outputs) start_writes(geom);
        ex_.allgather(send_.p, recv_.p, send_.n);
        pass_index_++;
    }

    // JointBilateralUpsampling of each owned view's previous-scale depth to
    // this scale's image (src/ACMMP.cpp:964-1087) on the device, kept there
    // for the hierarchy pass
    void jbu() {
        std::vector<int> views = mine_;
        views.insert(views.end(), split_.begin(), split_.end());
        for (int v : views) {
            ViewState &s = state_[v];
            const int id = problems_[(size_t)v].ref_image_id;
            const acmmp_camera &c = cams_.at(id);
            const size_t P = (size_t)s.W * s.H;
            DevBuf d(P);  // the depth channel of the previous scale's planes
            hip_check(hipMemcpy2DAsync(d.p, sizeof(float), s.planes.p + 3, 4 * sizeof(float), sizeof(float), P,
                                       hipMemcpyDeviceToDevice, copy_[0]),
                      "hipMemcpy2DAsync");
            hip_check(hipStreamSynchronize(copy_[0]), "hipStreamSynchronize");  // the JBU runs on its own stream
            s.jbu = DevBuf((size_t)c.width * c.height);
            int isc = 0;
            acmmp_check(acmmp_joint_bilateral_upsample_device(o_.device, images_.at(id).p, c.width, c.height, d.p, s.W,
                                                              s.H, s.jbu.p, &isc),
                        "acmmp_joint_bilateral_upsample_device");
            if (isc <= 1) fail("view " + std::to_string(id) + ": JBU image scale 1 (nothing to upsample)");
        }
    }

    VpOptions o_;
    Group &g_;
    Exchange ex_;
    std::string output_folder_;
    std::vector<acmmp_problem> problems_;
    std::map<int, int> index_of_;
    int max_down_ = -1;
    std::vector<std::vector<int>> assignment_;
    std::vector<int> mine_;   // views this rank computes whole
    std::vector<int> owned_;  // views whose image / depth slot and .dmb files are this rank's
    std::vector<int> split_;  // views every rank computes a band of
    bool split_checked_ = false;
    std::vector<acmmp_ctx *> engines_;
    std::vector<hipStream_t> copy_;  // per engine: the driver's device-to-device copies
    std::map<int, DevBuf> images_;
    std::map<int, acmmp_texture *> textures_;  // ~ the reference's texture objects, per image and scale
    std::map<int, acmmp_camera> cams_;
    std::vector<std::pair<int, int>> shape_;
    int slots_ = 1, hmax_ = 0, wmax_ = 0;
    DevBuf send_, recv_;
    DevBuf recv_img_;  // this scale's images of every view, gathered (textures borrow it)
    std::map<int, DevBuf> depth_tmp_;
    std::map<int, ViewState> state_;
    std::mutex mu_;
    int pass_index_ = 0;
    std::vector<std::thread> writers_;
    std::vector<std::string> write_errs_;
    std::map<std::string, double> phase_s_;
};

int env_int(const char *name, int dflt) {
    const char *v = std::getenv(name);
    return v && *v ? std::atoi(v) : dflt;
}

}  // namespace

int run_view_parallel(const VpOptions &opt) {
    try {
        const int rank = env_int("RANK", 0), world = env_int("WORLD_SIZE", 1);
        VpOptions o = opt;
        if (o.device < 0) o.device = env_int("LOCAL_RANK", 0);
        const char *addr = std::getenv("MASTER_ADDR");
        const int port = env_int("ACMMP_RDZV_PORT", env_int("MASTER_PORT", 29500) + 1);
        if (rank < 0 || world < 1 || rank >= world) fail("bad RANK / WORLD_SIZE");
        if (o.exchange_auto && world == 1) o.exchange_rccl = false;  // nothing to exchange
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        Group g(rank, world, addr && *addr ? addr : "127.0.0.1", port);
        double init_s = 0, run_s = 0;
        clk::time_point t3;
        {
            Driver d(o, g);  // problems, LPT, RCCL communicator, engines
            const auto t1 = clk::now();
            d.run();
            const auto t2 = clk::now();
            init_s = std::chrono::duration<double>(t1 - t0).count();
            run_s = std::chrono::duration<double>(t2 - t1).count();
            t3 = clk::now();
        }
        if (std::getenv("ACMMP_HOST_TIMING"))
            std::fprintf(stderr, "[rank %d] init=%.2fs run=%.2fs teardown=%.2fs\n", rank, init_s, run_s,
                         std::chrono::duration<double>(clk::now() - t3).count());
        if (rank == 0 && o.verbose)
            std::printf("view-parallel: %d ranks (%s exchange), maps under %s%s\n", world,
                        o.exchange_rccl ? "RCCL" : "TCP", o.dense.c_str(), o.output_dir.c_str());
        return 0;
    } catch (const std::exception &e) {
        std::fprintf(stderr, "acmmp_main --view_parallel: %s\n", e.what());
        return 1;
    }
}
