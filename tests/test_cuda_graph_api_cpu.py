"""The paddle.device.cuda.graphs namespace resolves under every reference spelling."""


def test_cuda_graphs_namespace():
    import paddle_infer_amd as paddle
    from paddle_infer_amd.device.cuda.graphs import CUDAGraph, wrap_cuda_graph, is_cuda_graph_supported
    from paddle_infer_amd.device.cuda import graphs
    assert paddle.device.cuda.graphs.CUDAGraph is CUDAGraph is graphs.CUDAGraph
    assert callable(wrap_cuda_graph)
    assert is_cuda_graph_supported() in (True, False)
