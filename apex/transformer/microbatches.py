"""Number-of-microbatches calculators (constant and linear batch-size ramp-up)."""
from __future__ import annotations


def build_num_microbatches_calculator(rank, rampup_batch_size, global_batch_size, micro_batch_size,
                                      data_parallel_size):
    if rampup_batch_size is None:
        return ConstantNumMicroBatches(global_batch_size, micro_batch_size, data_parallel_size)
    assert len(rampup_batch_size) == 3, "expected [start_batch_size, batch_size_increment, ramup_samples]"
    start, inc, samples = (int(x) for x in rampup_batch_size)
    return RampupBatchsizeNumMicroBatches(start, inc, samples, global_batch_size, micro_batch_size,
                                          data_parallel_size)


class NumMicroBatchesCalculator:
    def __init__(self):
        self.num_micro_batches = None
        self.current_global_batch_size = None

    def get(self):
        return self.num_micro_batches

    def get_current_global_batch_size(self):
        return self.current_global_batch_size

    def update(self, consumed_samples, consistency_check):
        pass


class ConstantNumMicroBatches(NumMicroBatchesCalculator):
    def __init__(self, global_batch_size, micro_batch_size, data_parallel_size):
        super().__init__()
        per = micro_batch_size * data_parallel_size
        assert global_batch_size % per == 0, (
            "global batch size ({}) is not divisible by micro batch size ({}) times data parallel size ({})"
            .format(global_batch_size, micro_batch_size, data_parallel_size))
        self.num_micro_batches = global_batch_size // per
        assert self.num_micro_batches >= 1
        self.current_global_batch_size = global_batch_size
        self.micro_batch_size = micro_batch_size


class RampupBatchsizeNumMicroBatches(NumMicroBatchesCalculator):
    def __init__(self, start_batch_size, batch_size_increment, ramup_samples, global_batch_size,
                 micro_batch_size, data_parallel_size):
        super().__init__()
        self.micro_batch_size = micro_batch_size
        self.data_parallel_size = data_parallel_size
        self.micro_batch_times_data_parallel_size = micro_batch_size * data_parallel_size
        self.start_batch_size = start_batch_size
        self.global_batch_size = global_batch_size
        diff = global_batch_size - start_batch_size
        assert diff >= 0 and diff % batch_size_increment == 0
        self.batch_size_increment = batch_size_increment
        self.rampup_samples_per_increment = ramup_samples / max(diff // batch_size_increment, 1)
        self.update(0, False)

    def update(self, consumed_samples, consistency_check):
        steps = int(consumed_samples / self.rampup_samples_per_increment)
        self.current_global_batch_size = min(self.start_batch_size + steps * self.batch_size_increment,
                                             self.global_batch_size)
        if consistency_check:
            assert self.current_global_batch_size % self.micro_batch_times_data_parallel_size == 0
        self.num_micro_batches = max(self.current_global_batch_size // self.micro_batch_times_data_parallel_size, 1)
