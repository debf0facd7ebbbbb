"""Error-feedback memories mirroring grace_dl/dist/memory/*.py."""
