"""Launchers: horovodrun-compatible elastic driver (hvdrun)."""
