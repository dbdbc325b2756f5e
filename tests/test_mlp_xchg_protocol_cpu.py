"""CPU emulation of the one-launch MLP's in-launch gradient exchange protocol (csrc/kernels/mlp_fused.hip
``xchg_tile`` on the xgmi_device.h primitives), VERDICT r5 next #7.

Ranks are threads; every launch of a rank runs its workgroups as threads joined at the launch end (the kernel
boundary).  Per launch: epoch = the rank's state epoch + 1 (read at workgroup start); workgroup b exchanges its
tile of layer j = nl-1 .. 0 (only the workgroups that own a tile of that layer) -- stage the value into slot
parity (epoch & 1) at the tile's offset, raise flag value epoch * nl + (nl-1-j) + 1 in EVERY rank's flag array at
[b][my rank], wait until every [b][r] flag of my array reached it, read all ranks' staged values in rank order; the
last workgroup to finish advances the state epoch.  Random delays everywhere and one slow reader: the other ranks
run ahead.  The emulation asserts every exchanged sum -- a slot overwritten by a later launch while still read would
break it; the control (test_emulation_detects_stale_flags) drops the epoch from the flag value, so a previous launch's
flag satisfies a wait, and the emulation reports the races."""
import random
import threading
import time


def _run(nranks=3, grid=6, tiles=(6, 4, 1), launches=7, seed=0):
    nl = len(tiles)
    off = [sum(tiles[:j]) for j in range(nl)]
    slots = [[[None] * sum(tiles) for _ in range(2)] for _ in range(nranks)]  # [rank][parity][tile]
    flags = [[[0] * nranks for _ in range(grid)] for _ in range(nranks)]       # [owner rank][b][writer rank]
    state = [{"epoch": 0, "done": 0} for _ in range(nranks)]
    locks = [threading.Lock() for _ in range(nranks)]
    errors = []
    rng = random.Random(seed)
    delays = [[rng.random() * 1e-4 for _ in range(64)] for _ in range(nranks)]

    def value(rank, launch, j, t):
        return (rank + 1) * 1000003 + launch * 1009 + j * 101 + t

    def workgroup(rank, launch, b, epoch):
        for j in range(nl - 1, -1, -1):
            if b >= tiles[j]:
                continue
            t = b
            idx = off[j] + t
            slots[rank][epoch & 1][idx] = value(rank, launch, j, t)
            v = epoch * nl + (nl - 1 - j) + 1
            time.sleep(delays[rank][(b + j) % 64])
            for r in range(nranks):  # publish: flag [b][my rank] in every rank's array
                flags[r][b][rank] = max(flags[r][b][rank], v)
            t0 = time.time()
            while any(flags[rank][b][r] < v for r in range(nranks)):  # wait (bounded)
                if time.time() - t0 > 20:
                    errors.append(("timeout", rank, launch, b, j))
                    return
                time.sleep(0)
            if rank == nranks - 1:
                time.sleep(5e-4)  # a slow reader (xgmi_read_delay): the others race ahead meanwhile
            vals = [slots[r][epoch & 1][idx] for r in range(nranks)]  # rank order
            if any(x is None for x in vals):
                errors.append(("unstaged", rank, launch, b, j))
                continue
            got = sum(vals)
            want = sum(value(r, launch, j, t) for r in range(nranks))
            if got != want:
                errors.append(("race", rank, launch, b, j, got, want))
        with locks[rank]:  # xgmi_finish: the last workgroup of the launch advances the epoch
            state[rank]["done"] += 1
            if state[rank]["done"] == grid:
                state[rank]["done"] = 0
                state[rank]["epoch"] = epoch

    def rank_main(rank):
        for launch in range(launches):
            epoch = state[rank]["epoch"] + 1  # every workgroup reads it at its start (before any finishes)
            ths = [threading.Thread(target=workgroup, args=(rank, launch, b, epoch)) for b in range(grid)]
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            time.sleep(delays[rank][launch % 64] * 3)

    ranks = [threading.Thread(target=rank_main, args=(r,)) for r in range(nranks)]
    for th in ranks:
        th.start()
    for th in ranks:
        th.join()
    return errors, state


def test_mlp_in_launch_exchange_protocol_emulated():
    for seed in range(4):
        errors, state = _run(seed=seed)
        assert not errors, errors[:5]
        assert all(s["epoch"] == 7 for s in state)


def test_mlp_exchange_flag_values_are_monotonic_per_workgroup():
    """The flag value of every (launch, exchange) pair of a workgroup is strictly larger than the previous one's,
    so a stale flag can never satisfy a later wait -- for any layer count and across launches."""
    for nl in range(1, 9):
        seq = [e * nl + (nl - 1 - j) + 1 for e in range(1, 6) for j in range(nl - 1, -1, -1)]
        assert all(b > a for a, b in zip(seq, seq[1:])), nl


def test_emulation_detects_stale_flags():
    """Control: flag values without the launch epoch (the same value every launch) let a wait pass on a previous
    launch's flag -- the emulation must report the resulting wrong sums."""
    src = open(__file__).read().replace("v = epoch * nl + (nl - 1 - j) + 1", "v = (nl - 1 - j) + 1")
    ns = {"__name__": "stale_flags"}
    exec(compile(src, __file__, "exec"), ns)
    races = sum(len(ns["_run"](seed=s, launches=5)[0]) for s in range(3))
    assert races > 0
