"""Device runtime: HIP stream pools (branch concurrency inside captured graphs), pinned host
staging rings with copy/compute/copy-back streams, and the hipGraph cache."""
