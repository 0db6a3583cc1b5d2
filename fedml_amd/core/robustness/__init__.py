from .robust_aggregation import RobustAggregator, is_weight_param, vectorize_weight, load_model_weight_diff

__all__ = ["RobustAggregator", "is_weight_param", "vectorize_weight", "load_model_weight_diff"]
