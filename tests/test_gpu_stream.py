"""Device IQ ring indexed by absolute sample count (gsdr_stream_*, SURVEY §8(b)
gsdr_stream_push / §8(f) rank 3): the stream pushed in GNU-Radio-sized chunks and
read in place by the acquisition grid (gsdr_acq_run_stream) and the tracking pool
(gsdr_trk_run_stream) gives results identical to the contiguous-buffer paths --
acquisition byte-identical to gsdr_acq_run on the same blocks, tracking records
identical to one contiguous gsdr_trk_run over the whole stream (the tracking
block consumes by nitems_read, dll_pll_veml_tracking.cc:1797,1818,2122, so a
call that needs items not pushed yet simply waits for the next push)."""
import numpy as np
import pytest
import torch

import gsdr
from gsdr import synth

pytestmark = pytest.mark.gpu

FS, N = 4000000, 4000


def _conf(nch, item=gsdr.ITEM_GR_COMPLEX):
    c = gsdr.trk_conf_default()
    c["fs_in"] = FS
    c["pll_bw_hz"] = 40.0
    c["dll_bw_hz"] = 4.0
    c["max_channels"] = nch
    c["item_type"] = item
    return c


def _acq_result(s):
    tau = s.code_delay_chips / 1.023e6 * FS
    return float(round(tau) % N), float(250 * round(s.doppler_hz / 250))


@pytest.mark.parametrize("item", [gsdr.ITEM_GR_COMPLEX, gsdr.ITEM_CSHORT])
def test_ring_matches_contiguous(item):
    ms = 160
    sats = synth.random_constellation(6, seed_offset=21)
    x = synth.gps_l1_iq(FS, ms * N, sats, seed_offset=21)
    if item == gsdr.ITEM_CSHORT:
        q = np.clip(np.rint(x.view(np.float32) * 40.0), -32767, 32767).astype(np.int16)
        items = q
        per_item = 2
    else:
        items = x
        per_item = 1
    codes = np.stack([synth.gps_ca_sampled(s.prn, FS) for s in sats])
    prns = np.array([s.prn for s in sats])
    acq = gsdr.Acquisition(FS, N, 10000, 250, pfa=0.01, max_prns=len(prns), item_type=item)
    acq.set_local_codes(codes, prns)
    # reference tracking: one contiguous run over the whole stream
    ref = gsdr.Tracking(_conf(len(sats), item))
    ring_trk = gsdr.Tracking(_conf(len(sats), item))
    for c, s in enumerate(sats):
        d, f = _acq_result(s)
        ref.start(c, s.prn, synth.gps_ca_chips(s.prn), d, f, 0, 0)
        ring_trk.start(c, s.prn, synth.gps_ca_chips(s.prn), d, f, 0, 0)
    ref_recs, ref_n = ref.run(items, 0, ms + 2)
    ring = gsdr.Stream(item, capacity_items=64 * N, max_window_items=40 * N)
    dev = torch.device("cuda", 0)
    me = 64
    out = torch.zeros(len(sats) * me * gsdr.TRK_EPOCH_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    nout = torch.zeros(len(sats), dtype=torch.int32, device=dev)
    got = [[] for _ in sats]
    acq_done = 0
    chunk = 4096
    pushed = 0
    total = ms * N
    while pushed < total:
        n = min(chunk, total - pushed)
        ring.push(items[pushed * per_item:(pushed + n) * per_item], pushed)
        pushed += n
        # acquisition of every block completed by this push, read in place
        while (acq_done + 1) * N <= pushed:
            b = acq_done
            r_ring = acq.run_stream(ring, b * N, 1, stamp0=(b + 1) * N)
            r_host = acq.run(items[b * N * per_item:(b + 1) * N * per_item], 1, stamp0=(b + 1) * N)
            assert r_ring.tobytes() == r_host.tobytes(), b
            acq_done += 1
        ring_trk.run_stream(ring, me, out.data_ptr(), nout.data_ptr())
        torch.cuda.synchronize(dev)
        recs = out.cpu().numpy().view(gsdr.TRK_EPOCH_DTYPE).reshape(len(sats), me)
        cnt = nout.cpu().numpy()
        for c in range(len(sats)):
            got[c].extend(recs[c, :cnt[c]].copy())
    assert acq_done == ms
    for c in range(len(sats)):
        g = np.array(got[c], dtype=gsdr.TRK_EPOCH_DTYPE)
        r = ref_recs[c, :ref_n[c]]
        assert len(g) == len(r) and len(g) >= ms - 2, (c, len(g), len(r))
        assert g.tobytes() == r.tobytes(), c
    ring.close()


def test_ring_errors():
    ring = gsdr.Stream(gsdr.ITEM_GR_COMPLEX, capacity_items=8 * N, max_window_items=4 * N)
    x = np.zeros(3 * N, np.complex64)
    ring.push(x, 1000)
    assert ring.span() == (1000, 3 * N)
    with pytest.raises(gsdr.GsdrError):
        ring.push(x, 5)  # not contiguous
    ring.push(x, 1000 + 3 * N)
    ring.push(x, 1000 + 6 * N)  # 9 N pushed, capacity 8 N: the oldest N dropped
    assert ring.span() == (1000 + 5 * N, 4 * N)
    with pytest.raises(gsdr.GsdrError):
        ring.window(1000, N)  # overwritten
    with pytest.raises(gsdr.GsdrError):
        ring.window(1000 + 2 * N, 5 * N)  # longer than the mirrored window
    assert ring.window(1000 + 4 * N, 4 * N)
    acq = gsdr.Acquisition(FS, N, 5000, 500, pfa=0.01, max_prns=1, item_type=gsdr.ITEM_CSHORT)
    acq.set_local_codes(synth.gps_ca_sampled(1, FS)[None], [1])
    with pytest.raises(gsdr.GsdrError):
        acq.run_stream(ring, 1000 + 5 * N, 1)  # item type mismatch
    ring.close()


def test_stalled_channel_reports_overrun():
    """A channel whose next call starts before the oldest item the ring still
    holds cannot continue: one record with LOSS_OF_LOCK | OVERRUN (event 3, the
    channel FSM re-acquires) and the channel in state 0, instead of a silent stall."""
    sats = synth.random_constellation(2, seed_offset=23)
    x = synth.gps_l1_iq(FS, 40 * N, sats, seed_offset=23)
    t = gsdr.Tracking(_conf(2))
    for c, s in enumerate(sats):
        d, f = _acq_result(s)
        t.start(c, s.prn, synth.gps_ca_chips(s.prn), d, f, 0, 0)
    ring = gsdr.Stream(gsdr.ITEM_GR_COMPLEX, capacity_items=8 * N, max_window_items=4 * N)
    pushed = 0
    while pushed < 40 * N:  # channels never run: the ring moves 32 ms past them
        ring.push(x[pushed:pushed + 2 * N], pushed)
        pushed += 2 * N
    rec, n = t.run_stream_host(ring, 16)
    for c in range(2):
        assert n[c] == 1, (c, n[c])
        assert rec[c, 0]["flags"] == gsdr.TRK_F_LOSS_OF_LOCK | gsdr.TRK_F_OVERRUN
        assert t.channel(c)["state"] == 0
    rec, n = t.run_stream_host(ring, 16)
    assert list(n) == [0, 0]
    ring.close()


def test_two_thread_push_and_consume():
    """GNU Radio deployment shape: a producer thread pushes while the consumer
    thread runs ring acquisitions and tracking; the ring lock held from window
    to reader event keeps every read identical to the contiguous-buffer result."""
    import threading
    ms = 96
    sats = synth.random_constellation(4, seed_offset=29)
    x = synth.gps_l1_iq(FS, ms * N, sats, seed_offset=29)
    codes = np.stack([synth.gps_ca_sampled(s.prn, FS) for s in sats])
    prns = np.array([s.prn for s in sats])
    acq = gsdr.Acquisition(FS, N, 10000, 250, pfa=0.01, max_prns=len(prns))
    acq.set_local_codes(codes, prns)
    ref_acq = acq.run(x, 1, stamp0=0)  # warm
    ring = gsdr.Stream(gsdr.ITEM_GR_COMPLEX, capacity_items=12 * N, max_window_items=4 * N)
    pushed = [0]
    cv = threading.Condition()
    stop = [False]

    def producer():
        while pushed[0] < ms * N:
            n = 1000
            with cv:
                # bounded lead over the consumer so the blocks it asks for are still held
                while pushed[0] - done[0] * N > 6 * N and not stop[0]:
                    cv.wait(0.05)
            ring.push(x[pushed[0]:pushed[0] + n], pushed[0])
            with cv:
                pushed[0] += n
                cv.notify_all()

    done = [0]
    th = threading.Thread(target=producer)
    th.start()
    try:
        while done[0] < ms:
            b = done[0]
            with cv:
                while pushed[0] < (b + 1) * N:
                    cv.wait(0.05)
            r_ring = acq.run_stream(ring, b * N, 1, stamp0=b * N)
            r_host = acq.run(x[b * N:(b + 1) * N], 1, stamp0=b * N)
            assert r_ring.tobytes() == r_host.tobytes(), b
            with cv:
                done[0] += 1
                cv.notify_all()
    finally:
        stop[0] = True
        th.join()
    assert ref_acq.shape == (1, len(prns))
    ring.close()


def test_async_window_blocks_overwrite():
    """gsdr_stream_window_async .. gsdr_stream_release with a producer thread: a push
    that would overwrite a window still open waits for its release, so every block
    read through the async window (acquisition on the consumer's own stream) equals
    the contiguous result even though the producer is allowed to run into the open
    block; a push over its own open window from the opening thread is refused
    (GSDR_E_STATE) and leaves the ring unchanged."""
    import threading
    import time
    ms = 40
    sats = synth.random_constellation(4, seed_offset=31)
    x = synth.gps_l1_iq(FS, (ms + 1) * N, sats, seed_offset=31)
    codes = np.stack([synth.gps_ca_sampled(s.prn, FS) for s in sats])
    prns = np.array([s.prn for s in sats])
    acq = gsdr.Acquisition(FS, N, 10000, 250, pfa=0.01, max_prns=len(prns))
    acq.set_local_codes(codes, prns)
    cap = 3 * N
    ring = gsdr.Stream(gsdr.ITEM_GR_COMPLEX, capacity_items=cap, max_window_items=N)
    cs = torch.cuda.Stream()
    rbytes = len(prns) * gsdr.ACQ_RESULT_DTYPE.itemsize
    res = torch.zeros(rbytes, dtype=torch.uint8, device="cuda")
    # the opening thread's own overwrite is refused
    ring.push(x[:cap], 0)
    ring.window_async(0, N, cs.cuda_stream)
    with pytest.raises(gsdr.GsdrError) as ei:
        ring.push(x[cap:cap + 1000], cap)
    assert ei.value.code == gsdr.GSDR_E_STATE
    ring.release(cs.cuda_stream)
    pushed = [cap]
    allowed = [0]  # the producer may overwrite samples below this
    cv = threading.Condition()

    def producer():
        while pushed[0] < ms * N:
            n = 1000
            with cv:
                while pushed[0] + n - cap > allowed[0]:
                    cv.wait(0.05)
            ring.push(x[pushed[0]:pushed[0] + n], pushed[0])  # may wait inside for a release
            with cv:
                pushed[0] += n
                cv.notify_all()

    th = threading.Thread(target=producer)
    th.start()
    try:
        for b in range(ms):
            with cv:
                while pushed[0] < (b + 1) * N:
                    cv.wait(0.05)
            p = ring.window_async(b * N, N, cs.cuda_stream)
            with cv:
                allowed[0] = (b + 1) * N  # block b itself is now guarded only by the open window
                cv.notify_all()
            time.sleep(0.002)  # let the producer run into the open window
            acq.run_device(p, 1, N, b * N, res.data_ptr(), stream_ptr=cs.cuda_stream)
            ring.release(cs.cuda_stream)
            cs.synchronize()
            got = res.cpu().numpy().view(gsdr.ACQ_RESULT_DTYPE).reshape(1, len(prns))
            ref = acq.run(x[b * N:(b + 1) * N], 1, stamp0=b * N)
            assert got.tobytes() == ref.tobytes(), b
    finally:
        ring.release(cs.cuda_stream)  # never leave the producer waiting on an open window
        with cv:
            allowed[0] = 1 << 62
            cv.notify_all()
        th.join()
    ring.close()
    acq.close()


def test_submit_collect_matches_contiguous():
    """gsdr_trk_submit_stream / gsdr_trk_collect (the pooled tracking blocks' advance):
    two submissions in flight while the next stretches are pushed (a push waits on the
    reader events of what it overwrites), the oldest polled without waiting, give
    records identical to one contiguous gsdr_trk_run; collect without a submission and
    a third submission in flight are refused."""
    ms = 120
    sats = synth.random_constellation(4, seed_offset=37)
    x = synth.gps_l1_iq(FS, ms * N, sats, seed_offset=37)
    ref = gsdr.Tracking(_conf(len(sats)))
    t = gsdr.Tracking(_conf(len(sats)))
    for c, s in enumerate(sats):
        d, f = _acq_result(s)
        ref.start(c, s.prn, synth.gps_ca_chips(s.prn), d, f, 0, 0)
        t.start(c, s.prn, synth.gps_ca_chips(s.prn), d, f, 0, 0)
    ref_recs, ref_n = ref.run(x, 0, ms + 2)
    ring = gsdr.Stream(gsdr.ITEM_GR_COMPLEX, capacity_items=32 * N, max_window_items=16 * N)
    with pytest.raises(gsdr.GsdrError):
        t.collect()
    got = [[] for _ in sats]

    def take(res):
        rec, n = res
        for c in range(len(sats)):
            got[c].extend(rec[c, :n[c]].copy())

    pushed, pending, polls = 0, 0, 0
    while pushed < ms * N:
        ring.push(x[pushed:pushed + 4 * N], pushed)
        pushed += 4 * N
        if pending == 2:
            res = t.collect(wait=False)
            polls += res is None
            if res is None:
                res = t.collect(wait=True)
            take(res)
            pending -= 1
        t.submit_stream(ring, 18)
        pending += 1
        if pending == 2 and pushed == 8 * N:
            with pytest.raises(gsdr.GsdrError):
                t.submit_stream(ring, 18)
    while pending:
        take(t.collect(wait=True))
        pending -= 1
    for c in range(len(sats)):
        g = np.array(got[c], dtype=gsdr.TRK_EPOCH_DTYPE)
        r = ref_recs[c, :ref_n[c]]
        assert len(g) == len(r) and len(g) >= ms - 2, (c, len(g), len(r))
        assert g.tobytes() == r.tobytes(), c
    ring.close()
