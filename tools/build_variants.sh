#!/bin/bash
# Rebuild the library and its diagnostic / A/B variants (run after any change to csrc/ or the
# header: a stale variant lacks symbols the binding table expects and fails to load).
set -e
cd "$(dirname "$0")/.."
python3 -c "import __graft_entry__ as g; g.build()"
python3 -c "from grace_amd.build import build; build(variant='stamps')"
GRACE_BUILD_DEFS=GRACE_TERN_FLUSH python3 -c "from grace_amd.build import build; build(variant='ternflush')"
GRACE_BUILD_DEFS=GRACE_TERN_ENC_NT python3 -c "from grace_amd.build import build; build(variant='ternnt')"
GRACE_BUILD_DEFS=GRACE_SEG_NOSMALL python3 -c "from grace_amd.build import build; build(variant='segnosmall')"
GRACE_BUILD_DEFS=GRACE_SEG_FIN_MULT=2 python3 -c "from grace_amd.build import build; build(variant='fin2k')"
