"""Distribution strategies, cluster resolution and collectives (tf.distribute surface)."""
from .cluster_resolver import ClusterSpec, TFConfigClusterResolver, TorchrunClusterResolver, SimpleClusterResolver  # noqa
from .strategy import (Strategy, OneDeviceStrategy, MirroredStrategy, MultiWorkerMirroredStrategy,  # noqa
                       ReduceOp, get_strategy, has_strategy, InputContext, CommunicationOptions,
                       CommunicationImplementation)
from .parameter_server import (ParameterServerStrategy, ParameterServer, run_parameter_server,  # noqa
                               ClusterCoordinator, partition)
from .kv import KVServer, KVClient  # noqa
