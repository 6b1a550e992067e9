"""Build an experimental variant of libmmt_hip.so with extra compile flags (A/B runs on the GPU box).

    python tools/build_variant.py NAME -DFOO=1 [...]
    MMT_LIB_PATH=build_variants/NAME/libmmt_hip.so python bench.py ...

Objects and the library go to build_variants/NAME/ (git-ignored; the tree ships to the GPU box).
"""
import concurrent.futures as cf
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "trade-aid-multimodal-transformer_amd"))
import mmt_build as B  # noqa: E402


def main():
    name, extra = sys.argv[1], sys.argv[2:]
    out = os.path.join(REPO, "build_variants", name)
    os.makedirs(out, exist_ok=True)

    def comp(src):
        o = os.path.join(out, src.replace(".hip", ".o"))
        r = subprocess.run([B.HIPCC] + B.FLAGS + B.FILE_FLAGS.get(src, []) + extra + ["-c", os.path.join(B.CSRC, src), "-o", o],
                           capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr)
        return o

    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(comp, B.SOURCES))
    lib = os.path.join(out, "libmmt_hip.so")
    subprocess.run([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib] + objs, check=True)
    print(lib)


if __name__ == "__main__":
    main()
