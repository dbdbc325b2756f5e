"""Gradient-bucket policy for RCCL over MI355X xGMI.

An MI355X node is a full mesh: every GPU has 7 point-to-point xGMI links (~153 GB/s each), so a
collective among ``w`` ranks can use ``min(w-1, 7)`` links per GPU, and a single ring uses only one.
RCCL spreads a buffer over its channels (several rings / direct peer transfers); each channel's slice
must stay well above the latency knee or the collective degenerates to a latency-bound chain of small
transfers.  That sets a *floor* on bucket size that grows with the number of active links, while
overlap with backward wants *several* buckets.  The reference relies on DDP's defaults (first bucket
1 MiB, then 25 MiB -- NVSwitch/PCIe-era numbers) and on Horovod's 64 MiB fusion buffer.

Policy (sizes in bytes of the reduced dtype):
* ``world == 1``: one bucket (no communication at all).
* floor = ``CHANNEL_MIN_BYTES * channels`` (channels = 2 per active link, or RCCL's pinned
  ``NCCL_MIN_NCHANNELS``) -- every channel's slice of every bucket is >= 256 KiB, so at world 8 each bucket
  splits into >= 14 channel-sized chunks over the 7 links (tests/test_ddp_cpu.py checks the plan); a
  trailing remainder below the floor is merged into the previous bucket.
* small models (total < 2 x floor, e.g. the 87 KB MNIST CNN, the 544 B hybrid fc): ONE bucket, reduced
  once after backward (latency-bound: a second collective would only add ~10-30 us of launch+sync).
* otherwise ``~4`` buckets (first one half-size so the last layer's gradients start moving early),
  each clamped to [floor, 64 MiB].
"""
from __future__ import annotations

import os

CHANNEL_MIN_BYTES = 256 * 1024
CHANNELS_PER_LINK = 2
MAX_BUCKET_BYTES = 64 * 1024 * 1024
TARGET_BUCKETS = 4


def active_links(world: int) -> int:
    return max(1, min(world - 1, 7))


def channels(world: int) -> int:
    """Channels the collective spreads a bucket over: RCCL's own minimum when the job pins it
    (``NCCL_MIN_NCHANNELS``), else ``CHANNELS_PER_LINK`` per active xGMI link."""
    env = os.environ.get("NCCL_MIN_NCHANNELS")
    if env and env.isdigit() and int(env) > 0:
        return max(int(env), active_links(world))
    return active_links(world) * CHANNELS_PER_LINK


def bucket_floor(world: int) -> int:
    return CHANNEL_MIN_BYTES * channels(world)


def plan_buckets(sizes_bytes: list[int], world: int, cap_bytes: int | None = None) -> list[list[int]]:
    """Group tensors (given in the order their gradients become ready) into buckets.

    Returns a list of buckets, each a list of tensor indices.  ``cap_bytes`` overrides the policy.
    """
    total = sum(sizes_bytes)
    if not sizes_bytes:
        return []
    if world <= 1 and cap_bytes is None:
        return [list(range(len(sizes_bytes)))]
    if cap_bytes is None:
        floor = bucket_floor(world)
        if total < 2 * floor:
            return [list(range(len(sizes_bytes)))]
        cap = min(MAX_BUCKET_BYTES, max(floor, total // TARGET_BUCKETS))
        first_cap = max(floor, cap // 2)
    else:
        cap = first_cap = max(1, cap_bytes)
        floor = 0
    buckets: list[list[int]] = []
    cur: list[int] = []
    cur_bytes = 0
    for i, b in enumerate(sizes_bytes):
        limit = first_cap if not buckets else cap
        if cur and cur_bytes + b > limit and cur_bytes >= floor:  # never close a bucket below the floor
            buckets.append(cur)
            cur, cur_bytes = [], 0
        cur.append(i)
        cur_bytes += b
    if cur:
        if buckets and cur_bytes < floor:
            buckets[-1].extend(cur)  # a remainder below the floor rides with the previous bucket
        else:
            buckets.append(cur)
    return buckets


def describe(world: int) -> str:
    return (f"xGMI bucket policy: world={world} active_links={active_links(world)} "
            f"floor={bucket_floor(world) / 2**20:.1f}MiB max={MAX_BUCKET_BYTES / 2**20:.0f}MiB")
