"""surfface_hip — host-side mirror of the surfface (matternet-rs) hot-path API
over the MI355X HIP C ABI (include/matternet_hip.h, libmatternet_hip.so).

Every op runs on the GPU through the C ABI; there is no CPU fallback.
"""
from . import _lib
from ._lib import MnError, lib
from . import clustering, energy, graph, l2f64, laplacian, search, sorted_index, sparsification
from .clustering import ClusteringOutput, ClusteringStage, nearest_centroid
from .graph import (BuilderParams, EigenMaps, GraphFactory, GraphLaplacian, SparsityError,
                    build_laplacian_matrix, standardize_columns)
from .l2f64 import (estimate_intrinsic_dimension, knn_l2_f64, nearest_subcentroid,
                    prepare_query_items_energy, topk_by_l2, topk_by_l2_rows)
from .search import (normalise_query_lambda, prepare_query_lambdas, search_lambda_aware,
                     search_lambda_aware_hybrid)
from .sparsification import SfGrassSparsifier, sparsify_rows, sparsify_sfgrass_csr
from .sorted_index import SortedLambdas
from .energy import (TauMode, compute_lambdas_gpu, compute_tau_mode_gpu, compute_taumode_lambdas,
                     diffuse_rows, energy_rows, laplacian_matvec_rows,
                     node_energy_and_dispersion, signal_energy_and_dispersion,
                     normalise_lambdas)
from .laplacian import (CsrMatrix, GraphParams, LaplacianConfig, LaplacianOutput, LaplacianStage,
                        build_laplacian_from_knn, compute_bhattacharyya_weights,
                        laplacian_stage_from_edges)
from .knn import (CandidateEdges, DistanceMetric, MSTConfig, ThicknessWeight, KnnResult, bf16_last_stats, build_candidate_graph, knn_cos_bf16,
                  knn_cos_bf16_qc, knn_cos_columns, knn_l2sq,
                  knn_l2sq_qc, last_stats, merge_parts)

__all__ = ["MnError", "lib", "clustering", "ClusteringOutput", "ClusteringStage",
           "nearest_centroid", "graph", "BuilderParams", "EigenMaps", "GraphFactory",
           "GraphLaplacian", "SparsityError", "build_laplacian_matrix", "standardize_columns", "knn_cos_columns", "knn_cos_bf16", "knn_cos_bf16_qc", "bf16_last_stats", "DistanceMetric", "MSTConfig", "ThicknessWeight", "CandidateEdges", "KnnResult", "build_candidate_graph", "knn_l2sq",
           "knn_l2sq_qc", "last_stats", "merge_parts", "CsrMatrix", "GraphParams",
           "LaplacianConfig", "LaplacianOutput", "build_laplacian_from_knn",
           "laplacian_stage_from_edges", "LaplacianStage", "compute_bhattacharyya_weights", "laplacian", "energy", "TauMode",
           "compute_taumode_lambdas", "energy_rows", "node_energy_and_dispersion",
           "compute_lambdas_gpu", "compute_tau_mode_gpu", "diffuse_rows",
           "laplacian_matvec_rows", "signal_energy_and_dispersion",
           "normalise_lambdas", "sorted_index", "SortedLambdas", "sparsification",
           "SfGrassSparsifier", "sparsify_rows", "sparsify_sfgrass_csr", "search", "search_lambda_aware",
           "normalise_query_lambda", "prepare_query_lambdas",
           "search_lambda_aware_hybrid", "l2f64", "knn_l2_f64", "topk_by_l2", "topk_by_l2_rows",
           "nearest_subcentroid", "prepare_query_items_energy", "estimate_intrinsic_dimension"]
