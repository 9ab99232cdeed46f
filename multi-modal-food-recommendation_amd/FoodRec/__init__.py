"""FoodRec on the MI355X engine.  Importing the package registers the engine's
torch_geometric.nn.GCNConv provider when torch_geometric itself is not installed (SCHGN's
``import torch_geometric`` then resolves; see FoodRec.engine.geometric)."""


def _install_graph_provider():
    from .engine import geometric
    geometric.install()


_install_graph_provider()
