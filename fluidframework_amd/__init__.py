"""fluidframework_amd — MI355X-native batch replay of Fluid merge-tree sequenced ops.

The one hot path of adrianlee/FluidFramework accelerated here is the observer replay of
sequenced merge-tree ops (``Client.applyMsg``, packages/dds/merge-tree/src/client.ts:797)
over many independent SharedString documents.  ``libmtreplay.so`` (csrc/, C ABI in
include/mtreplay.h) runs one wavefront per document on the GPU; this package is the
Python host layer over it.
"""
from .mtreplay import (  # noqa: F401
    EXPORTS,
    MT_BAD_INPUT,
    MT_CAPACITY,
    MT_ERR_NO_DEVICE,
    MT_INVALID_POS,
    MT_MSN_ORDER,
    MT_OK,
    MT_SEQ_ORDER,
    MT_UNSUPPORTED,
    DocView,
    GenParams,
    MtError,
    NotOnGpuPath,
    PackedJson,
    PackedJsonGpu,
    json_concat,
    ReplayBatch,
    gen_params,
    lib,
    status_string,
)
from .oplog import OP_DTYPE, PROP_DTYPE, Packer, PackedBatch, js_stringify, pack_documents  # noqa: F401

__all__ = ["ReplayBatch", "DocView", "GenParams", "gen_params", "Packer", "pack_documents", "lib"]
