"""Multi-process (world_size 2, gloo, CPU) coverage of the sharded path: block
and channel partitions tile the work, each rank runs the shard bench.rank_plan
gives it (the map bench.py and the engine launches use: one stream, block span
per rank, channels c % world) -- per-rank acquisition of its block span and
per-rank tracking of its channels (oracle restatement) merged on the host equal
the single-process results -- and the benchmark's barrier + max-over-ranks
timing reduction."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gsdr import shard, synth
from oracle import pcps

FS, N, DMAX, DSTEP = 2000000, 2000, 5000, 500
PRNS = (3, 7, 19)
BLOCKS_PER_RANK = 3
BLOCKS = 2 * BLOCKS_PER_RANK
TRK_CH = 3          # channels tracked (PRNS), sharded c % world
TRK_EPOCHS = 4


def _stream():
    sats = synth.random_constellation(3, seed_offset=7, cn0_dbhz=55.0, max_doppler=4000.0, prns=PRNS)
    return synth.gps_l1_iq(FS, BLOCKS * N, sats, seed_offset=7)


def _acq_blocks(x, lo, hi):
    D = int(np.ceil(2 * DMAX / DSTEP))
    wipe = pcps.doppler_wipeoffs(FS, N, DMAX, DSTEP, D)
    codes = [pcps.fft_code(synth.gps_ca_sampled(p, FS), N, N) for p in PRNS]
    out = np.zeros((hi - lo, len(PRNS), 3))
    for i, b in enumerate(range(lo, hi)):
        blk = x[b * N:(b + 1) * N]
        for k, c in enumerate(codes):
            ti, di, _, _, stat = pcps.max_to_input_power_statistic(pcps.magnitude_grid(blk, wipe, c))
            out[i, k] = (ti, di, stat)
    return out


def _track(x, channels):
    """Oracle tracking of the given channels over the stream (the engine's
    per-rank channel pool)."""
    from oracle import trk
    sats = synth.random_constellation(3, seed_offset=7, cn0_dbhz=55.0, max_doppler=4000.0, prns=PRNS)
    out = []
    for c in channels:
        s = sats[c]
        ch = trk.Channel(_trk_conf())
        tau = s.code_delay_chips / 1.023e6 * FS
        first = ch.start(synth.gps_ca_chips(s.prn), float(round(tau) % N), float(DSTEP * round(s.doppler_hz / DSTEP)),
                         0, 0)
        recs, _ = ch.run(x, 0, first, TRK_EPOCHS)
        out.append(np.array(recs["taps"][:, :6]).copy())
    return out


def _trk_conf():
    from oracle import trk
    c = np.zeros(1, trk.TRK_CONF_DTYPE)
    trk._lib().orc_trk_conf_default(c.ctypes.data)
    c["fs_in"] = FS
    c["max_channels"] = 1
    return c


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        x = _stream()
        plan = bench.rank_plan(world, rank, BLOCKS_PER_RANK, TRK_CH)
        assert plan["total_blocks"] == BLOCKS
        lo, hi = plan["blocks"]
        mine = torch.from_numpy(_acq_blocks(x, lo, hi))
        trk_mine = _track(x, plan["channels"])
        trk_all = [None] * world
        dist.all_gather_object(trk_all, trk_mine)
        # host-side result merge (object gather: spans differ in length)
        gathered = [None] * world
        dist.all_gather_object(gathered, mine.numpy())
        chans = shard.channels_of(12, world, rank).tolist()
        all_ch = [None] * world
        dist.all_gather_object(all_ch, chans)
        # bench.py: barrier, then max over ranks of the elapsed time
        dist.barrier()
        t = torch.tensor([1.0 + rank], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            q.put((gathered, all_ch, float(t.item()), trk_all))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_partitions_tile_the_work():
    for total in (0, 1, 5, 64, 1000):
        for world in (1, 2, 3, 8):
            spans = [shard.block_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
    for world in (1, 2, 8):
        ids = np.concatenate([shard.channels_of(256, world, r) for r in range(world)])
        assert sorted(ids.tolist()) == list(range(256))
    with pytest.raises(ValueError):
        shard.block_range(4, 2, 2)


def test_two_rank_gloo_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 2
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    os.environ["PYTHONPATH"] = os.pathsep.join([here, root, os.path.join(root, "gnss-sdr-new_amd"),
                                                os.environ.get("PYTHONPATH", "")])
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, all_ch, tmax, trk_all = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = shard.merge_blocks(gathered, BLOCKS, world)
    single = _acq_blocks(_stream(), 0, BLOCKS)
    np.testing.assert_array_equal(merged[..., :2], single[..., :2])
    np.testing.assert_allclose(merged[..., 2], single[..., 2], rtol=0, atol=0)
    assert sorted(sum(all_ch, [])) == list(range(12))
    assert tmax == 2.0
    recs = shard.merge_channels([[("r0", c) for c in all_ch[0]], [("r1", c) for c in all_ch[1]]], 12, world)
    assert [r[1] for r in recs] == list(range(12))
    # tracking: channel c on rank c % 2, merged == one process tracking every channel
    merged_trk = shard.merge_channels(trk_all, TRK_CH, world)
    single_trk = _track(_stream(), list(range(TRK_CH)))
    for a, b in zip(merged_trk, single_trk):
        assert a.shape == (TRK_EPOCHS, 6)
        np.testing.assert_array_equal(a, b)


def _c5_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        plan = bench.c5_rank_plan(world, rank, 8)
        plans = [None] * world
        dist.all_gather_object(plans, plan)
        dist.barrier()
        t = torch.tensor([0.5 + rank], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            q.put((plans, float(t.item())))
    finally:
        dist.destroy_process_group()


def test_c5_plan_tiles_the_job():
    """bench.py --workload c5 (BASELINE C5: 256 hybrid channels over the node's
    GPUs): at every world size the ranks' block spans tile the stream, the 256
    channels land once each on rank c % world in three signal pools, each rank's
    acquisition grids cover its span (GPS / BeiDou on alternate ms, Galileo per
    4 ms group), and the per-rank work stays constant (weak scaling)."""
    import bench
    work = set()
    for world in (1, 2, 4, 8):
        plans = [bench.c5_rank_plan(world, r, 8) for r in range(world)]
        spans = [p["blocks"] for p in plans]
        assert spans[0][0] == 0 and spans[-1][1] == 8 * world
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
        chans = sorted(sum((p["channels"] for p in plans), []))
        assert chans == list(range(256))
        for r, p in enumerate(plans):
            assert all(c % world == r for c in p["channels"])
            assert sorted(sum(p["pools"].values(), [])) == p["channels"]
            lo, hi = p["blocks"]
            a = p["acq"]
            assert sorted(a["gps_blocks"] + a["bds_blocks"]) == list(range(lo, hi))
            assert [g for g in a["gal_groups"]] == list(range(lo, hi, 4))
            # per-rank work: grids, channel-milliseconds of tracking
            work.add((len(a["gps_blocks"]), len(a["bds_blocks"]), len(a["gal_groups"]),
                      len(p["channels"]) * p["total_blocks"]))
        if world == 8:
            assert all([len(p["pools"][s]) for s in (0, 1, 2)] == [12, 12, 8] for p in plans)
    assert len(work) == 1
    with pytest.raises(ValueError):
        bench.c5_rank_plan(2, 0, 6)


def test_c5_plan_two_rank_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    os.environ["PYTHONPATH"] = os.pathsep.join([here, root, os.path.join(root, "gnss-sdr-new_amd"),
                                                os.environ.get("PYTHONPATH", "")])
    port = _free_port()
    procs = [ctx.Process(target=_c5_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    plans, tmax = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == 1.5
    assert sorted(plans[0]["channels"] + plans[1]["channels"]) == list(range(256))
    assert plans[0]["blocks"] == (0, 8) and plans[1]["blocks"] == (8, 16)


class _StubEngine:
    """CPU stand-in for the gsdr engine calls of bench.main's C2 path: the same
    Python API (gsdr.Acquisition / gsdr.Tracking), recording each launch instead of
    running it.  Rank 1's launches take longer, so the max over ranks is visible."""

    def __init__(self, log, rank):
        import gsdr
        self._log, self._rank = log, rank
        self.ACQ_RESULT_DTYPE, self.TRK_EPOCH_DTYPE = gsdr.ACQ_RESULT_DTYPE, gsdr.TRK_EPOCH_DTYPE
        self.synth = synth
        eng = self

        class Acquisition:
            def __init__(self, fs, n, dmax, dstep, max_blocks=1, **kw):
                self.n, self.max_blocks, self.wipe_mode, self.spectrum_reuse = n, max_blocks, 0, (4, 16)

            def set_local_codes(self, codes, prns):
                eng._log.append(("codes", len(prns)))

            def run_device(self, iq_ptr, nblocks, stride, stamp0, res_ptr, stream=None):
                assert 0 < nblocks <= self.max_blocks
                eng._log.append(("acq", int(stamp0) // self.n, int(nblocks)))
                import time
                time.sleep(0.002 * (1 + eng._rank))

            def set_profiling(self, on):
                pass

            def close(self):
                pass

        class Tracking:
            def __init__(self, conf, device=0):
                self.nch = int(conf["max_channels"][0])

            def start(self, ch, prn, code, delay, dop, stamp, nread):
                eng._log.append(("trk_start", int(ch), int(prn)))

            def save_state(self, slot):
                pass

            def restore_state(self, slot):
                pass

            def run_device(self, iq_ptr, first, items, max_epochs, out_ptr, n_ptr, stream=None):
                eng._log.append(("trk", int(max_epochs)))

            def set_profiling(self, on):
                pass

            def close(self):
                pass

        self.Acquisition, self.Tracking = Acquisition, Tracking

    def trk_conf_default(self):
        import gsdr
        return np.zeros(1, gsdr.TRK_CONF_DTYPE)


def _bench_worker(rank, world, port, q):
    """One rank of `bench.py --gpus 2` under torch.distributed.run, the device calls
    stubbed: bench.main itself does the process-group init (gloo instead of RCCL),
    the barriers around the timed region and the max-over-ranks time."""
    import contextlib
    import io
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    log = []

    class CpuBackend:
        dist_backend = "gloo"

        def __init__(self, local):
            self.torch, self.dev = torch, torch.device("cpu")
            self.gsdr = _StubEngine(log, rank)

        def dist_kwargs(self):
            return {}

        def synchronize(self):
            pass

        def event(self):
            raise AssertionError("no profile events in this rehearsal")

    out = io.StringIO()
    try:
        with contextlib.redirect_stdout(out):
            bench.main(["--gpus", str(world), "--steps", "3", "--warmup", "1", "--no-profile-events",
                        "--no-cpu-baseline", "--min-warmup-ms", "0"], backend=CpuBackend)
    except BaseException as e:  # report instead of leaving the parent waiting
        q.put((rank, None, repr(e)))
        raise
    q.put((rank, log, out.getvalue()))


def test_bench_main_two_rank_gloo_control_flow():
    """bench.py's real C2 control flow at world size 2 with the device calls stubbed
    (tests the multi-rank path before an 8-GPU measurement): each rank acquires its
    own block span of the one stream every step and tracks channels c % 2; rank 0
    prints the one JSON line, whose value is all ranks' samples over the slowest
    rank's time."""
    import json
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    os.environ["PYTHONPATH"] = os.pathsep.join([here, root, os.path.join(root, "gnss-sdr-new_amd"),
                                                os.environ.get("PYTHONPATH", "")])
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, (log, out)) for r, log, out in (q.get(timeout=240), q.get(timeout=240)))
    assert all(v[0] is not None for v in got.values()), got
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import bench
    line = json.loads(got[0][1].strip().splitlines()[-1])
    assert got[1][1].strip() == ""  # only rank 0 prints
    assert line["n_gpus"] == 2 and line["steps"] == 3 and line["scaling"] == "weak"
    B = line["config"]["blocks_per_step"]
    # all ranks' samples over the max-over-ranks time: rank 1 (slower) sets it
    assert abs(line["value"] - 2 * 3 * B * bench.N / (line["ms_per_step"] * 3e-3) / 1e6) <= 1e-3 * line["value"]
    assert line["ms_per_step"] >= 2 * 0.002 * 2 * 1e3 * 0.9  # rank 1's two chains sleep 4 ms per step
    total = 2 * B
    for r in (0, 1):
        log = got[r][0]
        lo, hi = bench.rank_plan(2, r, B, bench.CHANNELS)["blocks"]
        acq = [e for e in log if e[0] == "acq"]
        # two chains x (1 warmup + 3 timed steps + 3 steps of the acquisition-only rate)
        assert len(acq) == 2 * 7
        for s in range(4):
            spans = sorted((e[1] - s * total, e[2]) for e in acq[2 * s:2 * s + 2])
            assert spans[0][0] == lo and spans[0][0] + spans[0][1] == spans[1][0] and spans[1][0] + spans[1][1] == hi
        mine = bench.rank_plan(2, r, B, bench.CHANNELS)["channels"]
        assert [e[1] for e in log if e[0] == "trk_start"] == list(range(len(mine)))
        assert all(c % 2 == r for c in mine) and len(mine) == bench.CHANNELS // 2
        # one tracking launch for the warmup, one for the timed steps, one for the tracking-only rate
        assert [e for e in log if e[0] == "trk"] == [("trk", 1 * total), ("trk", 3 * total), ("trk", 3 * total)]


def test_bench_acq_stagger_tiles_each_step(monkeypatch):
    """`bench.py --acq-stagger S` (round 6): the two chains take B/2 + S and B/2 - S blocks
    on alternate steps, and every step's two launches still tile the step's B blocks."""
    import contextlib
    import io
    import json
    import bench
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    log = []

    class CpuBackend:
        dist_backend = "gloo"

        def __init__(self, local):
            self.torch, self.dev = torch, torch.device("cpu")
            self.gsdr = _StubEngine(log, 0)

        def dist_kwargs(self):
            return {}

        def synchronize(self):
            pass

        def event(self):
            raise AssertionError("no profile events here")

    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        bench.main(["--steps", "3", "--warmup", "1", "--no-profile-events", "--no-cpu-baseline", "--acq-stagger", "8",
                    "--min-warmup-ms", "0"], backend=CpuBackend)
    line = json.loads(out.getvalue().strip().splitlines()[-1])
    B = line["config"]["blocks_per_step"]
    assert line["config"]["acq_stagger"] == 8
    acq = [e for e in log if e[0] == "acq"]
    assert len(acq) == 2 * 7  # (1 warmup + 3 timed + 3 acquisition-only) steps x two chains
    for s in range(7):
        a, b = acq[2 * s], acq[2 * s + 1]
        step = s if s < 4 else s - 4  # the acquisition-only rate restarts at step 0
        first = B // 2 + 8 if step % 2 == 0 else B // 2 - 8
        assert (a[2], b[2]) == (first, B - first)
        span = (s if s < 4 else s - 4) * B
        assert a[1] - span == 0 and b[1] - span == a[2]


def test_bench_clock_warmup_precedes_the_warmup_steps():
    """--min-warmup-ms (round 6): untimed acquisition passes for at least that long before
    the W warmup steps; the timed region still runs exactly K steps."""
    import time
    import bench
    calls, syncs = [], []
    n = bench.clock_warmup(lambda k: (calls.append(k), time.sleep(0.001)), 30.0, lambda: syncs.append(len(calls)))
    assert n == len(calls) >= 10 and calls == list(range(n))
    assert syncs == [4]  # one synchronised burst sizes a pass; the rest run back to back
    assert bench.clock_warmup(lambda k: calls.append(k), 0.0, lambda: None) == 0
