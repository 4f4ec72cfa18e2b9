// host_pool.cpp -- the process-wide host worker pool of the host-batch paths.
//
// The segment-list gathers and scatters (nfec_*_host_vectors: NORM's scattered segment pool,
// normSegment.cpp:14-86), the strided staging copies (nfec_*_host) and the large host repairs
// split their bytes over host threads.  A codec striped over N GPUs runs N such pipelines at
// once (one driver thread per device), so per-call thread spawns would put
// N x (threads per call) gather threads on the job's cores -- 64 on a 16-core cgroup share at
// N = 8.  Instead every call queues its pieces on one pool of host_pool_size() workers, the
// cores the job may actually use (affinity mask capped by the cgroup cpu.max quota, as
// bench.py's host_cores does), so the copies of all stripes together never run on more threads
// than that.  The callers (device drivers, mostly waiting on the GPU) hand their pieces to the
// pool and wait; a pool worker that calls in (none does today) runs its pieces inline.
#include "nfec_internal.hpp"

#include <sched.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>

namespace nfec {

namespace {

unsigned cgroup_quota_cores()
{
    // cgroup v2: "<quota> <period>" or "max <period>"
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[64] = {0};
        unsigned long long period = 0;
        const int got = std::fscanf(f, "%63s %llu", q, &period);
        std::fclose(f);
        if (got == 2 && std::strcmp(q, "max") != 0 && period > 0) {
            const unsigned long long quota = std::strtoull(q, nullptr, 10);
            return (unsigned)std::max<unsigned long long>(1, quota / period);
        }
    }
    return 0;  // no quota
}

struct PoolJob {
    std::function<void(unsigned)> fn;
    std::atomic<unsigned> next{0};
    unsigned n = 0;
    std::mutex mu;
    std::condition_variable cv;
    unsigned done = 0;  // pieces finished, thrown or not (under mu)
    int err = NFEC_OK;  // the first piece that threw (under mu)
    std::string what;
};

// runs piece i; an exception (std::bad_alloc in a piece's allocation, anything else a piece
// throws) is caught here -- a worker thread must not terminate the process and the caller must
// not wait forever -- and reported as a status: NFEC_ENOMEM for bad_alloc, NFEC_EINVAL otherwise
int run_piece(const std::function<void(unsigned)>& fn, unsigned i, std::string& what)
{
    try {
        fn(i);
        return NFEC_OK;
    } catch (const std::bad_alloc&) {
        what = "host pool piece: out of memory";
        return NFEC_ENOMEM;
    } catch (const std::exception& e) {
        what = std::string("host pool piece: ") + e.what();
        return NFEC_EINVAL;
    } catch (...) {
        what = "host pool piece: unknown exception";
        return NFEC_EINVAL;
    }
}

thread_local bool tl_pool_worker = false;
std::atomic<unsigned> g_active{0}, g_max_active{0};  // pool pieces running now / at most so far

class HostPool {
  public:
    explicit HostPool(unsigned workers) : pid_(getpid())
    {
        for (unsigned i = 0; i < workers; ++i) {
            try {
                th_.emplace_back([this] { loop(); });
            } catch (...) {
                break;  // fewer workers than planned (none: the callers run their pieces inline)
            }
        }
    }
    unsigned workers() const { return (unsigned)th_.size(); }

    // NFEC_OK, or the status of the first piece that threw (every piece runs either way)
    int run(unsigned n, const std::function<void(unsigned)>& fn)
    {
        if (n == 0) return NFEC_OK;
        // inline: one piece, no workers, a call from a worker, or a child forked after the pool
        // started (it inherits the pool object but not its threads, and a queue lock a thread
        // held at the fork would stay held: the child never touches the queue)
        if (n == 1 || th_.empty() || tl_pool_worker || getpid() != pid_) {
            int err = NFEC_OK;
            std::string what;
            for (unsigned i = 0; i < n; ++i) {
                std::string w;
                const int rc = run_piece(fn, i, w);
                if (rc && !err) err = rc, what = w;
            }
            return err ? fail(err, what) : NFEC_OK;
        }
        auto job = std::make_shared<PoolJob>();
        job->fn = fn;
        job->n = n;
        {
            std::lock_guard<std::mutex> lk(mu_);
            // one queue entry per worker that can help (each entry drains pieces until none is left)
            for (unsigned i = 0; i < std::min(n, workers()); ++i) q_.push_back(job);
        }
        cv_.notify_all();
        std::unique_lock<std::mutex> lk(job->mu);
        job->cv.wait(lk, [&] { return job->done == job->n; });
        return job->err ? fail(job->err, job->what) : NFEC_OK;
    }

  private:
    void loop()
    {
        tl_pool_worker = true;
        for (;;) {
            std::shared_ptr<PoolJob> job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return !q_.empty(); });
                job = std::move(q_.front());
                q_.pop_front();
            }
            for (;;) {
                const unsigned i = job->next.fetch_add(1);
                if (i >= job->n) break;
                const unsigned a = g_active.fetch_add(1) + 1;
                unsigned mx = g_max_active.load();
                while (a > mx && !g_max_active.compare_exchange_weak(mx, a)) {
                }
                std::string what;
                const int rc = run_piece(job->fn, i, what);
                g_active.fetch_sub(1);
                std::lock_guard<std::mutex> lk(job->mu);
                if (rc && !job->err) job->err = rc, job->what = what;
                if (++job->done == job->n) job->cv.notify_all();
            }
        }
    }
    const pid_t pid_;  // the process that started the workers
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<PoolJob>> q_;
};

HostPool& pool()
{
    // created on first use and never destroyed: its workers outlive every codec (static
    // destruction order at exit would otherwise race with codecs destroyed late)
    static HostPool* p = new HostPool(host_pool_size());
    return *p;
}

}  // namespace

unsigned host_visible_cores()
{
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(set), &set) == 0) return std::max(1, CPU_COUNT(&set));
    return std::max(1u, std::thread::hardware_concurrency());
}

unsigned host_usable_cores()
{
    const unsigned vis = host_visible_cores(), quota = cgroup_quota_cores();
    return quota ? std::min(vis, quota) : vis;
}

unsigned host_pool_size()
{
    static const unsigned n = [] {
        unsigned t = host_usable_cores();
        if (const char* v = std::getenv("NFEC_HOST_THREADS")) t = (unsigned)std::max(1, std::atoi(v));
        return std::min<unsigned>(t, 64);
    }();
    return n;
}

int host_parallel_for(unsigned n, const std::function<void(unsigned)>& fn) { return pool().run(n, fn); }

unsigned host_pool_workers() { return pool().workers(); }

unsigned host_pool_max_active(bool reset)
{
    return reset ? g_max_active.exchange(0) : g_max_active.load();
}

}  // namespace nfec
