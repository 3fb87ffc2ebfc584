// vdb/metric.h — distance metric ordinals of the reference (engine/kernels.cuh:24-28),
// without any device headers. L2 = squared L2, InnerProduct = negated dot product,
// Cosine = the reference CPU path's behaviour (distance 0.0f, ivf_flat_index.cpp:351-362).
#pragma once

namespace vdb {
namespace kernels {
enum class Metric { L2, InnerProduct, Cosine };
}  // namespace kernels
}  // namespace vdb
