"""The library stamp a profile was measured with.

Every profile file bench.py embeds (profiles/rNN/pmc_traffic.json,
step_flops_pmc.json) carries `smmd_source_hash`: the SHA-256 stamp of the
csrc/ sources + header (gan.core._lib.source_hash, the string csrc/Makefile
compiles into libsmmd_hip.so and _lib.lib() checks at load).  bench.py embeds
such a file only when its stamp equals the running library's."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scaled-mmd-gan_amd'))


def library_stamp():
    """{'smmd_source_hash': stamp of the tree's sources, 'library_has_stamp':
    whether the built .so embeds that same string} (no GPU, no HIP call)."""
    from gan.core import _lib
    stamp = _lib.source_hash()
    try:
        with open(_lib.LIB_PATH, 'rb') as f:
            has = stamp.encode() in f.read()
    except OSError:
        has = False
    return {'smmd_source_hash': stamp, 'library_has_stamp': has}


if __name__ == '__main__':
    print(library_stamp())
