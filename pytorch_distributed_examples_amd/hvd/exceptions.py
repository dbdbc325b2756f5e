"""Horovod-compatible exception types (horovod.common.exceptions)."""


class HorovodInternalError(RuntimeError):
    """A collective failed (e.g. a peer died); elastic ``run`` restores the last commit and resets."""


class HostsUpdatedInterrupt(RuntimeError):
    """The elastic driver reported a membership change; raised from ``State.commit()``.

    ``skip_sync`` is True when hosts were only removed (surviving state is already consistent)."""

    def __init__(self, skip_sync: bool = False):
        super().__init__("hosts updated")
        self.skip_sync = skip_sync
