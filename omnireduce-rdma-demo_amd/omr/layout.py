"""Block/lane/partition layout of the reference (common.h:27-42), as a value object.

Vocabulary:
  n               DATA_SIZE floats (common.h:40)
  block_size      BLOCK_SIZE floats per block (common.h:32)
  num_threads     NUM_THREADS partitions, each DATA_SIZE_PER_THREAD = n/num_threads floats (common.h:35, :38)
  num_lanes       NUM_BLOCKS = NUM_SLOTS*MESSAGE_SIZE/BLOCK_SIZE (common.h:36-37): lane bid = block % num_lanes
  row             num_lanes consecutive blocks; a partition holds rows_per_part rows
  sentinel        (UINT32_MAX/B/NB - 1)*NB*B (client.cc:24); lane l's end marker is sentinel + l*B
"""
from __future__ import annotations

from dataclasses import dataclass

UINT32_MAX = 0xFFFFFFFF
MESSAGE_SIZE = 1024  # common.h:31
NUM_SLOTS = 16  # common.h:36 (8*NUM_QPS*2)
NUM_THREADS = 8  # common.h:35


@dataclass(frozen=True)
class Layout:
    n: int
    block_size: int = 256
    num_threads: int = NUM_THREADS
    message_size: int = MESSAGE_SIZE
    num_slots: int = NUM_SLOTS

    def __post_init__(self):
        if self.block_size <= 0 or self.message_size % self.block_size:
            raise ValueError(f"BLOCK_SIZE {self.block_size} must divide MESSAGE_SIZE {self.message_size}")
        if self.n % (self.num_threads * self.row_floats):
            raise ValueError(f"n={self.n} is not a multiple of NUM_THREADS*NUM_BLOCKS*BLOCK_SIZE="
                             f"{self.num_threads * self.row_floats}")
        if self.n > self.sentinel:
            raise ValueError(f"n={self.n} exceeds the uint32 offset space (sentinel {self.sentinel})")

    @classmethod
    def from_bytes(cls, nbytes: int, block_size: int = 256, num_threads: int = NUM_THREADS) -> "Layout":
        return cls(n=nbytes // 4, block_size=block_size, num_threads=num_threads)

    @property
    def blocks_per_message(self) -> int:  # common.h:33
        return self.message_size // self.block_size

    @property
    def num_lanes(self) -> int:  # NUM_BLOCKS, common.h:37
        return self.num_slots * self.blocks_per_message

    @property
    def row_floats(self) -> int:
        return self.num_lanes * self.block_size

    @property
    def data_size_per_thread(self) -> int:  # common.h:38
        return self.n // self.num_threads

    @property
    def nb(self) -> int:  # BITMAP_SIZE, common.h:42
        return self.n // self.block_size

    @property
    def rows(self) -> int:
        return self.nb // self.num_lanes

    @property
    def rows_per_part(self) -> int:
        return self.rows // self.num_threads

    @property
    def nbytes(self) -> int:
        return self.n * 4

    @property
    def sentinel(self) -> int:  # client.cc:24 / server.cc:16, uint32 arithmetic
        nbl = self.num_slots * self.message_size // self.block_size
        return ((UINT32_MAX // self.block_size // nbl - 1) * nbl * self.block_size) & UINT32_MAX

    def lane_of(self, offset: int) -> int:  # client.cc:23
        return (offset // self.block_size) % self.num_lanes

    def partition_of(self, offset: int) -> int:
        return offset // self.data_size_per_thread

    def head_offset(self, tid: int, bid: int) -> int:  # client.cc:43 start_offset + i*BLOCK_SIZE
        return tid * self.data_size_per_thread + bid * self.block_size

    def global_slot(self, tid: int, slot: int) -> int:  # common.cc:381-383: gs = slot + NUM_SLOTS*tid
        return slot + self.num_slots * tid
