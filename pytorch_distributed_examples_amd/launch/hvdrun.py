"""Elastic launcher / driver with ``horovodrun``'s CLI surface (reference usage at
horovod/horovod_mnist_elastic.py:108):

    python -m pytorch_distributed_examples_amd.launch.hvdrun -np 2 --min-np 1 --max-np 8 \
        --blacklist-cooldown-range 15 30 --host-discovery-script ./discover_hosts.sh \
        horovod/horovod_mnist_elastic.py [script args]

The driver hosts a c10d TCPStore and publishes membership *rounds* (:mod:`..elastic.rendezvous`).  Workers
are processes on this node, one per discovered slot (``host:slots`` lines from the discovery script or
``-H``); on an MI355X node each gets its own GPU (LOCAL_RANK).

* worker exits non-zero  -> its host is blacklisted for a random cooldown in the given range, a new round
  with the survivors is published (>= --min-np), survivors catch the failed collective
  (HorovodInternalError), restore their last commit and re-rendezvous IN-PROCESS;
* discovery finds new slots -> new workers are spawned, a new round is published and the running workers
  see ``updated/<round>`` at their next ``state.commit()`` (HostsUpdatedInterrupt);
* discovery drops a host -> its workers are terminated and the survivors re-rendezvous;
* all workers exit 0 -> the job succeeds.

Multi-node ssh spawning is out of scope for this single-node build (workers of every discovered "host"
run locally); the rendezvous protocol itself is host-agnostic.
"""
from __future__ import annotations

import argparse
import datetime
import os
import random
import signal
import subprocess
import sys
import time

import torch.distributed as dist

from ..parallel.dist import free_port


def parse_hosts(text: str, default_slots: int) -> list[tuple[str, int]]:
    hosts = []
    for tok in text.replace(",", "\n").split():
        tok = tok.strip()
        if not tok:
            continue
        if ":" in tok:
            h, s = tok.rsplit(":", 1)
            hosts.append((h, int(s)))
        else:
            hosts.append((tok, default_slots))
    return hosts


def run_discovery(script: str, default_slots: int) -> list[tuple[str, int]]:
    try:
        out = subprocess.run([script], capture_output=True, text=True, timeout=30, shell=False)
    except Exception as exc:  # noqa: BLE001
        print(f"[hvdrun] discovery script failed: {exc}", file=sys.stderr, flush=True)
        return []
    if out.returncode != 0:
        return []
    return parse_hosts(out.stdout, default_slots)


class Worker:
    def __init__(self, wid, host, slot, device, proc):
        self.wid, self.host, self.slot, self.device, self.proc = wid, host, slot, device, proc
        self.finished = False


class Driver:
    def __init__(self, args, command):
        self.args = args
        self.command = command
        self.port = free_port()
        self.store = dist.TCPStore("127.0.0.1", self.port, is_master=True,
                                   timeout=datetime.timedelta(seconds=args.start_timeout), wait_for_workers=False)
        self.round = -1
        self.workers: dict[str, Worker] = {}
        self.order: list[str] = []  # rank order of the current round
        self.blacklist: dict[str, float] = {}
        self.counter = 0
        self.free_devices = list(range(args.num_devices)) if args.num_devices > 0 else []
        self.leaving: dict[str, float] = {}  # worker id -> deadline of a planned departure

    # ---------------------------------------------------------------------------------------------
    def log(self, msg):
        if self.args.verbose:
            print(f"[hvdrun] {msg}", flush=True)

    def discovered_slots(self) -> list[tuple[str, int]]:
        if self.args.host_discovery_script:
            hosts = run_discovery(self.args.host_discovery_script, self.args.slots_per_host)
        elif self.args.hosts:
            hosts = parse_hosts(self.args.hosts, self.args.slots_per_host)
        else:
            hosts = [("localhost", self.args.np)]
        now = time.time()
        slots = []
        for h, n in hosts:
            if self.blacklist.get(h, 0) > now:
                continue
            slots.extend((h, i) for i in range(n))
        return slots

    def spawn(self, host: str, slot: int) -> Worker:
        wid = f"{host}:{slot}:{self.counter}"
        self.counter += 1
        dev = self.free_devices.pop(0) if self.free_devices else slot
        env = dict(os.environ)
        env.update({"PDE_ELASTIC_STORE": f"127.0.0.1:{self.port}", "PDE_WORKER_ID": wid, "LOCAL_RANK": str(dev),
                    "PDE_HOST": host, "HOROVOD_HOSTNAME": host, "OMP_NUM_THREADS": env.get("OMP_NUM_THREADS", "1")})
        proc = subprocess.Popen(self.command, env=env)
        w = Worker(wid, host, slot, dev, proc)
        self.workers[wid] = w
        self.log(f"spawned {wid} (pid {proc.pid}, device {dev})")
        return w

    def alive(self) -> list[Worker]:
        return [w for w in self.workers.values() if w.proc.poll() is None]

    def publish(self, members: list[str]):
        if self.round >= 0:
            self.store.set(f"updated/{self.round}", "1")
        r = self.round + 1
        self.store.set(f"round/{r}/size", str(len(members)))
        self.store.set(f"round/{r}/members", ",".join(members))  # rank order (shrink detection)
        for rank, wid in enumerate(members):
            self.store.set(f"round/{r}/rank/{wid}", str(rank))
        self.store.set("round", str(r))
        self.round = r
        self.order = list(members)
        self.log(f"round {r}: size {len(members)} members {members}")

    def release(self, w: Worker):
        if w.device not in self.free_devices and self.args.num_devices > 0:
            self.free_devices.append(w.device)
            self.free_devices.sort()

    # ---------------------------------------------------------------------------------------------
    def run(self) -> int:
        slots = self.discovered_slots()
        target = min(self.args.max_np, max(self.args.np, 0) or len(slots), len(slots))
        if target < self.args.min_np:
            print(f"[hvdrun] only {len(slots)} slots available, need >= {self.args.min_np}", file=sys.stderr)
            return 1
        for h, s in slots[:target]:
            self.spawn(h, s)
        self.publish([w.wid for w in self.workers.values()])
        last_discovery = time.time()
        deadline = None
        while True:
            time.sleep(0.1)
            changed = False
            for w in list(self.workers.values()):
                rc = w.proc.poll()
                if rc is None or w.finished:
                    continue
                w.finished = True
                self.release(w)
                if rc == 0:
                    self.log(f"{w.wid} finished")
                    continue
                lo, hi = self.args.blacklist_cooldown_range
                cool = random.uniform(lo, hi) if hi > 0 else 0.0
                self.blacklist[w.host] = time.time() + cool
                print(f"[hvdrun] worker {w.wid} failed (exit {rc}); blacklisting host {w.host} for {cool:.1f}s",
                      flush=True)
                if w.wid in self.order:
                    changed = True
                    # report the failure of this round's member AT ONCE (survivors abort their spinning xGMI
                    # exchanges on it: elastic/rewire.py _FailureWatch); the new round follows below
                    failed = [x for x in self.order if self.workers[x].finished and self.workers[x].proc.returncode]
                    self.store.set(f"failed/{self.round}", ",".join(failed))
            for wid, dl in list(self.leaving.items()):
                if self.workers[wid].proc.poll() is not None:
                    del self.leaving[wid]
                elif time.time() > dl:
                    self.log(f"{wid} did not leave within {self.args.leave_grace}s: terminating")
                    self.workers[wid].proc.send_signal(signal.SIGTERM)
                    del self.leaving[wid]
            members = [wid for wid in self.order if self.workers[wid].proc.poll() is None]
            if all(w.finished for w in self.workers.values()):
                ok = all(w.proc.returncode == 0 for w in self.workers.values() if w.wid in self.order) or \
                    any(w.proc.returncode == 0 for w in self.workers.values())
                self.store.set("shutdown", "1")
                return 0 if ok else 1
            # discovery: add / remove workers
            if (time.time() - last_discovery >= self.args.discovery_interval or changed) and \
                    (self.args.host_discovery_script or changed):
                last_discovery = time.time()
                slots = self.discovered_slots()
                used = {(self.workers[wid].host, self.workers[wid].slot) for wid in members}
                allowed_hosts = {h for h, _ in slots}
                for wid in list(members):
                    if self.workers[wid].host not in allowed_hosts and self.args.host_discovery_script:
                        # a PLANNED scale-down: the worker sees the new round at its next commit point, takes
                        # part in the communicator split (rewire.RoundComm.planned_split) and exits 0;
                        # terminated only if it has not left within --leave-grace seconds
                        self.log(f"host of {wid} removed by discovery: asking it to leave")
                        self.leaving[wid] = time.time() + self.args.leave_grace
                        members.remove(wid)
                        changed = True
                if any(self.workers[wid].finished and self.workers[wid].proc.returncode == 0
                       for wid in self.order):
                    pass  # job is finishing: do not grow
                else:
                    for h, s in slots:
                        if len(members) >= self.args.max_np:
                            break
                        if (h, s) not in used:
                            members.append(self.spawn(h, s).wid)
                            used.add((h, s))
                            changed = True
            if changed:
                if len(members) < self.args.min_np:
                    if deadline is None:
                        deadline = time.time() + self.args.elastic_timeout
                        print(f"[hvdrun] {len(members)} < min-np {self.args.min_np}: waiting for hosts", flush=True)
                    if time.time() > deadline:
                        self.store.set("shutdown", "1")
                        for w in self.alive():
                            w.proc.terminate()
                        return 1
                    continue
                deadline = None
                self.publish(members)


def main(argv=None):
    ap = argparse.ArgumentParser(description="horovodrun-compatible elastic launcher (single node)")
    ap.add_argument("-np", "--num-proc", dest="np", type=int, default=0)
    ap.add_argument("--min-np", type=int, default=None)
    ap.add_argument("--max-np", type=int, default=None)
    ap.add_argument("-H", "--hosts", default=None)
    ap.add_argument("--host-discovery-script", default=None)
    ap.add_argument("--slots-per-host", "--slots", type=int, default=1)
    ap.add_argument("--blacklist-cooldown-range", type=float, nargs=2, default=(0.0, 0.0))
    ap.add_argument("--discovery-interval", type=float, default=1.0)
    ap.add_argument("--start-timeout", type=float, default=600.0)
    ap.add_argument("--elastic-timeout", type=float, default=600.0)
    ap.add_argument("--leave-grace", type=float, default=60.0,
                    help="seconds a worker whose host discovery dropped may take to leave by itself (it joins the "
                         "communicator split at its next commit point) before it is terminated")
    ap.add_argument("--num-devices", type=int, default=-1, help="GPUs on this node (default: autodetect)")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("command", nargs=argparse.REMAINDER)
    args = ap.parse_args(argv)
    if not args.command:
        ap.error("missing training command")
    cmd = args.command
    if cmd[0].endswith(".py"):
        cmd = [sys.executable] + cmd
    if args.np <= 0 and not (args.hosts or args.host_discovery_script):
        args.np = 1
    args.min_np = args.min_np if args.min_np is not None else max(1, args.np)
    args.max_np = args.max_np if args.max_np is not None else max(args.np, 1 << 16)
    if args.num_devices < 0:
        try:
            import torch

            args.num_devices = torch.cuda.device_count()
        except Exception:  # noqa: BLE001
            args.num_devices = 0
    sys.exit(Driver(args, cmd).run())


if __name__ == "__main__":
    main()
