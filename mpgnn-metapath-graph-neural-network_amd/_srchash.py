"""Source hash of libmpgnn_rgcn.so (no package imports: __graft_entry__.build() loads this file
by path before the library exists). build() writes it next to the library; _lib.py refuses a
library whose stamp does not match the sources in the tree."""
import hashlib
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = ("csrc/Makefile", "csrc/plan.cpp", "csrc/plan_internal.h", "csrc/io.cpp", "csrc/rgcn_kernels.hip",
           "csrc/plan_device.hip", "csrc/score_kernels.hip", "csrc/optim_kernels.hip", "../include/mpgnn_rgcn.h")
STAMP = os.path.join(HERE, "libmpgnn_rgcn.so.srchash")


def source_hash() -> str:
    """sha256 over the files csrc/Makefile compiles and includes."""
    h = hashlib.sha256()
    for rel in SOURCES:
        with open(os.path.join(HERE, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read() + b"\0")
    return h.hexdigest()


def sources_present() -> bool:
    return all(os.path.exists(os.path.join(HERE, r)) for r in SOURCES)


def write_stamp() -> str:
    h = source_hash()
    with open(STAMP, "w") as f:
        f.write(h + "\n")
    return h


if __name__ == "__main__":  # csrc/Makefile: after every library link
    print("source hash", write_stamp()[:16])
