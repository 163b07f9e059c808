// Device IQ ring indexed by absolute sample count (SURVEY §8(b) gsdr_stream_push,
// §8(f) rank 3, §7 H6): the input stream is uploaded once per GPU and every
// consumer -- the acquisition grid, the tracking channel pool -- reads its window
// in place by absolute sample index, the index dll_pll_veml_tracking itself uses
// (nitems_read, dll_pll_veml_tracking.cc:1797,1818,2122) and pcps_acquisition's
// sample stamp counts (pcps_acquisition.cc:968,1009).
//
// Layout: `cap` items at ring positions sample % cap, plus a mirror of the first
// `window` positions after the end, so any window of up to `window` items is one
// contiguous device span (no consumer handles the wrap).  Pushes run on the
// ring's own copy stream; a consumer launch waits on the last push's event and
// records a reader event of its own, tagged with the oldest item it reads; a push
// waits only for the readers whose oldest item it overwrites.  Consumers on other
// streams (the tracking pools of several signals, the acquisition services) thus
// run concurrently with each other and with the pushes of newer items.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "gsdr_internal.h"
#include "gsdr_stream_internal.h"

struct gsdr_stream
{
    int device{0};
    int item_type{GSDR_ITEM_GR_COMPLEX};
    size_t item_bytes{8};
    uint64_t cap{0};     // ring positions
    uint64_t window{0};  // longest contiguous window (mirrored positions)
    uint8_t* d_ring{nullptr};
    bool started{false};
    uint64_t base{0};  // absolute index of the first item pushed
    uint64_t head{0};  // absolute index of the next item to push
    hipStream_t copy{nullptr};
    hipEvent_t pushed{nullptr};
    // consumer launches that may still read the ring: the oldest item each reads and
    // the event recorded behind it on its stream
    struct Reader
    {
        uint64_t lo;
        hipEvent_t ev;
    };
    std::vector<Reader> readers;
    // pushes whose copies may still read the caller's host memory: the absolute end
    // of each and the event recorded behind its copies, oldest first
    struct Pending
    {
        uint64_t end;
        hipEvent_t ev;
    };
    std::vector<Pending> pending;
    uint64_t landed{0};  // every item before it is in device memory
    std::vector<hipEvent_t> retired;  // waited for by a push, recycled once complete
    std::vector<hipEvent_t> spare;
    // windows handed out by gsdr_stream_window_async whose reads are not yet
    // released: a push that would overwrite one waits for its release (another
    // thread's window) or fails (the pushing thread's own window)
    struct OpenWindow
    {
        hipStream_t consumer;
        uint64_t first;
        std::thread::id owner;
    };
    std::vector<OpenWindow> open;
    std::condition_variable released;
    std::mutex mu;
};

namespace gsdr
{
int stream_item_type(const gsdr_stream* s) { return s->item_type; }
int stream_device(const gsdr_stream* s) { return s->device; }

namespace
{
uint64_t oldest_of(const gsdr_stream* s) { return s->head > s->cap ? std::max(s->base, s->head - s->cap) : s->base; }

// (ring lock held)
int view_locked(gsdr_stream* s, uint64_t first, uint64_t n, const void** ptr)
{
    GSDR_REQUIRE(s->started, GSDR_E_STATE, "gsdr_stream: nothing pushed yet");
    const uint64_t oldest = oldest_of(s);
    GSDR_REQUIRE(first >= oldest && first + n <= s->head, GSDR_E_ARG,
        "gsdr_stream: window [%llu, %llu) outside the ring's [%llu, %llu)", (unsigned long long)first,
        (unsigned long long)(first + n), (unsigned long long)oldest, (unsigned long long)s->head);
    GSDR_REQUIRE(n <= s->window, GSDR_E_ARG, "gsdr_stream: window of %llu items exceeds the ring's %llu",
        (unsigned long long)n, (unsigned long long)s->window);
    *ptr = s->d_ring + (first % s->cap) * s->item_bytes;
    return GSDR_OK;
}

int span_locked(gsdr_stream* s, uint64_t* first, uint64_t* n)
{
    GSDR_REQUIRE(s->started, GSDR_E_STATE, "gsdr_stream: nothing pushed yet");
    const uint64_t oldest = oldest_of(s);
    const uint64_t lo = s->head > s->window ? std::max(oldest, s->head - s->window) : oldest;
    *first = lo;
    *n = s->head - lo;
    return GSDR_OK;
}

// reader events that completed go back to the spare list (ring lock held)
void recycle_locked(gsdr_stream* s)
{
    auto done = [s](hipEvent_t ev) {
        if (hipEventQuery(ev) != hipSuccess) return false;
        s->spare.push_back(ev);
        return true;
    };
    s->readers.erase(std::remove_if(s->readers.begin(), s->readers.end(),
                         [&](const gsdr_stream::Reader& r) { return done(r.ev); }),
        s->readers.end());
    s->retired.erase(std::remove_if(s->retired.begin(), s->retired.end(), done), s->retired.end());
}

// pushes whose copies completed leave `pending` (their events to the spare list);
// wait: block until every push holding an item before `upto` completed (ring lock held)
int land_locked(gsdr_stream* s, bool wait, uint64_t upto)
{
    size_t k = 0;
    for (; k < s->pending.size(); ++k)
        {
            const gsdr_stream::Pending& p = s->pending[k];
            if (wait && s->landed < upto)  // s->landed: this push's first item
                GSDR_HIP(hipEventSynchronize(p.ev));
            else
                {
                    const hipError_t q = hipEventQuery(p.ev);
                    if (q == hipErrorNotReady) break;
                    GSDR_HIP(q);
                }
            s->landed = p.end;
            s->spare.push_back(p.ev);
        }
    s->pending.erase(s->pending.begin(), s->pending.begin() + static_cast<std::ptrdiff_t>(k));
    if (s->pending.empty()) s->landed = s->head;
    return GSDR_OK;
}

// the consumer's reads of items >= lo are enqueued on `consumer`: a push that
// overwrites any of them waits for the event recorded here
int release_locked(gsdr_stream* s, hipStream_t consumer, uint64_t lo)
{
    if (s->readers.size() + s->retired.size() >= 16) recycle_locked(s);
    hipEvent_t ev = nullptr;
    if (!s->spare.empty())
        {
            ev = s->spare.back();
            s->spare.pop_back();
        }
    else
        GSDR_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const hipError_t e = hipEventRecord(ev, consumer);
    if (e != hipSuccess)
        {
            s->spare.push_back(ev);
            GSDR_HIP(e);
        }
    s->readers.push_back({lo, ev});
    return GSDR_OK;
}
}  // namespace

StreamReader::StreamReader(gsdr_stream* s) : s_(s), lk_(s->mu) {}
int StreamReader::view(uint64_t first, uint64_t n, const void** ptr)
{
    const int rc = view_locked(s_, first, n, ptr);
    if (rc == GSDR_OK) lo_ = std::min(lo_, first);
    return rc;
}
int StreamReader::span(uint64_t* first, uint64_t* n) { return span_locked(s_, first, n); }
int StreamReader::acquire(hipStream_t consumer)
{
    // a push that already landed needs no cross-queue dependency (a barrier packet on
    // the consumer's queue waiting for the copy engine's signal delays the launch)
    const hipError_t q = hipEventQuery(s_->pushed);
    if (q == hipSuccess) return GSDR_OK;
    if (q != hipErrorNotReady) GSDR_HIP(q);
    GSDR_HIP(hipStreamWaitEvent(consumer, s_->pushed, 0));
    return GSDR_OK;
}
int StreamReader::release(hipStream_t consumer) { return release_locked(s_, consumer, lo_ == UINT64_MAX ? 0 : lo_); }
}  // namespace gsdr

namespace
{
size_t bytes_of(int it) { return it == GSDR_ITEM_CSHORT ? 4 : (it == GSDR_ITEM_IBYTE ? 2 : 8); }
}  // namespace

extern "C" {

int gsdr_stream_create(int device, int item_type, uint64_t capacity_items, uint64_t max_window_items, gsdr_stream** out)
{
    GSDR_REQUIRE(out, GSDR_E_ARG, "gsdr_stream_create: null argument");
    *out = nullptr;
    GSDR_REQUIRE(item_type >= GSDR_ITEM_GR_COMPLEX && item_type <= GSDR_ITEM_IBYTE, GSDR_E_ARG,
        "gsdr_stream_create: unknown item type %d", item_type);
    GSDR_REQUIRE(capacity_items > 0 && max_window_items > 0 && max_window_items <= capacity_items, GSDR_E_ARG,
        "gsdr_stream_create: need 0 < max_window_items <= capacity_items");
    int ndev = 0;
    GSDR_HIP(hipGetDeviceCount(&ndev));
    GSDR_REQUIRE(device >= 0 && device < ndev, GSDR_E_ARG, "gsdr_stream_create: device %d of %d", device, ndev);
    gsdr::DeviceGuard g(device);
    auto* s = new (std::nothrow) gsdr_stream();
    GSDR_REQUIRE(s, GSDR_E_ALLOC, "gsdr_stream_create: out of host memory");
    s->device = device;
    s->item_type = item_type;
    s->item_bytes = bytes_of(item_type);
    s->cap = capacity_items;
    s->window = max_window_items;
    hipError_t e = hipMalloc(&s->d_ring, (size_t)(s->cap + s->window) * s->item_bytes);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->copy, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s->pushed, hipEventDisableTiming);
    if (e != hipSuccess)
        {
            gsdr::set_error("gsdr_stream_create: %s", hipGetErrorString(e));
            gsdr_stream_destroy(s);
            return GSDR_E_ALLOC;
        }
    *out = s;
    return GSDR_OK;
}

void gsdr_stream_destroy(gsdr_stream* s)
{
    if (!s) return;
    gsdr::DeviceGuard g(s->device);
    if (s->copy) (void)hipStreamSynchronize(s->copy);
    for (const auto& r : s->readers)
        {
            (void)hipEventSynchronize(r.ev);
            (void)hipEventDestroy(r.ev);
        }
    for (hipEvent_t ev : s->retired)
        {
            (void)hipEventSynchronize(ev);
            (void)hipEventDestroy(ev);
        }
    for (const auto& p : s->pending) (void)hipEventDestroy(p.ev);  // the copy stream drained above
    for (hipEvent_t ev : s->spare) (void)hipEventDestroy(ev);
    if (s->pushed) (void)hipEventDestroy(s->pushed);
    if (s->copy) (void)hipStreamDestroy(s->copy);
    if (s->d_ring) (void)hipFree(s->d_ring);
    delete s;
}

int gsdr_stream_push(gsdr_stream* s, const void* iq_host, uint64_t first_sample, uint64_t n)
{
    GSDR_REQUIRE(s && (iq_host || n == 0), GSDR_E_ARG, "gsdr_stream_push: null argument");
    std::unique_lock<std::mutex> lk(s->mu);
    gsdr::DeviceGuard g(s->device);
    if (!s->started)
        {
            s->started = true;
            s->base = s->head = s->landed = first_sample;
        }
    GSDR_REQUIRE(n <= s->cap, GSDR_E_ARG, "gsdr_stream_push: %llu items exceed the ring capacity %llu",
        (unsigned long long)n, (unsigned long long)s->cap);
    // samples below new_oldest lose their ring positions: an async window still
    // open over them must be released first (its reads are not enqueued yet, so
    // the reader event cannot cover them).  The wait drops the lock, so the head
    // (another pusher) and the windows are re-read after every wakeup; a window
    // left open for kStallLimit (a consumer that failed before its release) ends
    // the push with GSDR_E_STATE instead of hanging it.
    constexpr auto kStallLimit = std::chrono::seconds(10);
    const auto deadline = std::chrono::steady_clock::now() + kStallLimit;
    for (;;)
        {
            GSDR_REQUIRE(first_sample == s->head, GSDR_E_ARG,
                "gsdr_stream_push: items must be contiguous (next is %llu, got %llu)", (unsigned long long)s->head,
                (unsigned long long)first_sample);
            if (n == 0) return GSDR_OK;
            const uint64_t new_oldest = s->head + n > s->cap ? s->head + n - s->cap : 0;
            bool blocked = false;
            for (const auto& w : s->open)
                if (w.first < new_oldest)
                    {
                        GSDR_REQUIRE(w.owner != std::this_thread::get_id(), GSDR_E_STATE,
                            "gsdr_stream_push: would overwrite the window at %llu this thread holds open "
                            "(gsdr_stream_window_async); release it first", (unsigned long long)w.first);
                        blocked = true;
                    }
            if (!blocked) break;
            GSDR_REQUIRE(s->released.wait_until(lk, deadline) != std::cv_status::timeout, GSDR_E_STATE,
                "gsdr_stream_push: a window over the items it would overwrite stayed open for %lld s "
                "(gsdr_stream_release missing)", (long long)kStallLimit.count());
        }
    // overwrite only what no consumer launch still reads: the copy waits for the
    // readers of items below the new oldest (later pushes are ordered behind it)
    const uint64_t overwritten = s->head + n > s->cap ? s->head + n - s->cap : 0;
    for (auto it = s->readers.begin(); it != s->readers.end();)
        {
            if (it->lo < overwritten)
                {
                    GSDR_HIP(hipStreamWaitEvent(s->copy, it->ev, 0));
                    s->retired.push_back(it->ev);
                    it = s->readers.erase(it);
                }
            else
                ++it;
        }
    const auto* src = static_cast<const uint8_t*>(iq_host);
    uint64_t done = 0;
    while (done < n)
        {
            const uint64_t pos = (s->head + done) % s->cap;
            const uint64_t len = std::min<uint64_t>(n - done, s->cap - pos);
            GSDR_HIP(hipMemcpyAsync(s->d_ring + pos * s->item_bytes, src + done * s->item_bytes, len * s->item_bytes,
                hipMemcpyHostToDevice, s->copy));
            if (pos < s->window)
                {
                    // mirror of the first `window` positions after the end
                    const uint64_t mlen = std::min<uint64_t>(len, s->window - pos);
                    GSDR_HIP(hipMemcpyAsync(s->d_ring + (s->cap + pos) * s->item_bytes, src + done * s->item_bytes,
                        mlen * s->item_bytes, hipMemcpyHostToDevice, s->copy));
                }
            done += len;
        }
    GSDR_HIP(hipEventRecord(s->pushed, s->copy));
    // the push's own event: iq_host is the caller's until it completes
    if (s->pending.size() >= 64)
        {
            const int rc = gsdr::land_locked(s, false, 0);
            if (rc != GSDR_OK) return rc;
        }
    hipEvent_t ev = nullptr;
    if (!s->spare.empty())
        {
            ev = s->spare.back();
            s->spare.pop_back();
        }
    else
        GSDR_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const hipError_t e = hipEventRecord(ev, s->copy);
    if (e != hipSuccess)
        {
            s->spare.push_back(ev);
            GSDR_HIP(e);
        }
    s->head += n;
    s->pending.push_back({s->head, ev});
    return GSDR_OK;
}

int gsdr_stream_landed(gsdr_stream* s, uint64_t* landed)
{
    GSDR_REQUIRE(s && landed, GSDR_E_ARG, "gsdr_stream_landed: null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    gsdr::DeviceGuard g(s->device);
    const int rc = gsdr::land_locked(s, false, 0);
    *landed = s->landed;
    return rc;
}

int gsdr_stream_wait_landed(gsdr_stream* s, uint64_t upto)
{
    GSDR_REQUIRE(s, GSDR_E_ARG, "gsdr_stream_wait_landed: null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    gsdr::DeviceGuard g(s->device);
    return gsdr::land_locked(s, true, upto);
}

int gsdr_stream_span(gsdr_stream* s, uint64_t* first_sample, uint64_t* n_items)
{
    GSDR_REQUIRE(s && first_sample && n_items, GSDR_E_ARG, "gsdr_stream_span: null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    return gsdr::span_locked(s, first_sample, n_items);
}

int gsdr_stream_window(gsdr_stream* s, uint64_t first_sample, uint64_t n_items, const void** iq_dev)
{
    GSDR_REQUIRE(s && iq_dev, GSDR_E_ARG, "gsdr_stream_window: null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    int rc = gsdr::view_locked(s, first_sample, n_items, iq_dev);
    if (rc != GSDR_OK) return rc;
    gsdr::DeviceGuard g(s->device);
    GSDR_HIP(hipEventSynchronize(s->pushed));
    return GSDR_OK;
}

int gsdr_stream_window_async(gsdr_stream* s, uint64_t first_sample, uint64_t n_items, void* consumer_stream,
    const void** iq_dev)
{
    GSDR_REQUIRE(s && consumer_stream && iq_dev, GSDR_E_ARG, "gsdr_stream_window_async: null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    int rc = gsdr::view_locked(s, first_sample, n_items, iq_dev);
    if (rc != GSDR_OK) return rc;
    gsdr::DeviceGuard g(s->device);
    GSDR_HIP(hipStreamWaitEvent((hipStream_t)consumer_stream, s->pushed, 0));
    s->open.push_back({(hipStream_t)consumer_stream, first_sample, std::this_thread::get_id()});
    return GSDR_OK;
}

int gsdr_stream_release(gsdr_stream* s, void* consumer_stream)
{
    GSDR_REQUIRE(s && consumer_stream, GSDR_E_ARG, "gsdr_stream_release: null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    gsdr::DeviceGuard g(s->device);
    const hipStream_t c = (hipStream_t)consumer_stream;
    // the oldest item of the windows this consumer holds open (none: every item)
    uint64_t lo = UINT64_MAX;
    for (const auto& w : s->open)
        if (w.consumer == c) lo = std::min(lo, w.first);
    if (lo == UINT64_MAX) lo = 0;
    const int rc = gsdr::release_locked(s, c, lo);
    // the reader event now covers this consumer's reads: its windows close
    s->open.erase(std::remove_if(s->open.begin(), s->open.end(), [c](const gsdr_stream::OpenWindow& w) {
        return w.consumer == c;
    }), s->open.end());
    s->released.notify_all();
    return rc;
}

int gsdr_stream_device(const gsdr_stream* s, int* device)
{
    GSDR_REQUIRE(s && device, GSDR_E_ARG, "gsdr_stream_device: null argument");
    *device = s->device;
    return GSDR_OK;
}

}  // extern "C"
