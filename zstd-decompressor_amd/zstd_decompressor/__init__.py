"""MI355X-native mirror of the `zstd_decompressor` crate API
(AchilleBailly/zstd-decompressor, zstd-decompressor/src/lib.rs:2-9).

Module map (reference -> here):
  parsing.rs          -> parsing       ForwardByteParser, FrameIterator entry
  frame.rs            -> frame         Frame, ZStandard, Skippable, Header, FrameIterator
  block.rs            -> block         Block.parse / Block.decode(ctx)
  decoding_context.rs -> decoding_context  DecodingContext (GPU-resident)
  decoders/, literals.rs, sequences.rs -> HIP kernels behind the C ABI (include/zd.h)
Batch API (the hot path): batch.decompress / batch.Plan.
"""
from . import _lib
from ._lib import ZdError
from .parsing import ForwardByteParser
from .frame import Frame, FrameIterator, Header, Skippable, ZStandard, MAX_WIN_SIZE
from .block import Block
from .decoding_context import DecodingContext
from .batch import Plan, decompress, frames_index

__all__ = ["ZdError", "ForwardByteParser", "Frame", "FrameIterator", "Header", "Skippable", "ZStandard",
           "MAX_WIN_SIZE", "Block", "DecodingContext", "Plan", "decompress", "frames_index"]
