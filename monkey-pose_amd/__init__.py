"""monkey-pose_amd: MI355X (gfx950) inference path of krg-nandu/monkey-pose's 3D pose regressors.

The directory name carries a hyphen, so import it with ``importlib.import_module("monkey-pose_amd")``
(see ``tests/conftest.py``).  Modules:

* ``hgru_pose``   -- drop-in ``model().build(depth, output_shape)`` (reference ``hgru_pose.py``)
* ``hgru_module`` -- drop-in ``ContextualCircuit(X, ...).build()`` (reference ``hgru_module.py``)
* ``train_dense_networks.dense_model_struct`` / ``train_hier_networks.hier_model_struct`` --
  drop-ins for the dense and hierarchical regressor heads
* ``train_dense_hier_networks.dense_hier_model_struct`` -- the dense-hierarchical hybrid, recorded
  as a layer graph (``_graph``) and run by the native graph runtime (``mp_graph_*``)
* ``train_cnn_networks_hgru`` -- ``attn_model_struct`` (the attention CoM regressor),
  ``prepare_data_test`` (device batch crop) and ``FramePosePipeline`` (frame -> CoM -> crop -> pose)
* ``monkeydetector`` -- ``MonkeyDetector`` / ``tfMonkeyDetector``: CoM, crop (native), joint transforms
* ``pose_evaluation`` -- the host metrics (``getMeanError_np`` ...)
* ``weights``     -- TF variable-name tables and deterministic synthetic initialisers
* ``tf_checkpoint`` -- TF1 V2 checkpoint reader / writer (no TensorFlow needed)
* ``data_loader`` -- TFRecord ingestion (``inputs`` / ``read_and_decode``, ``create_tf_record``)
* ``_lib``        -- ctypes binding of ``libmonkeypose.so`` (C ABI: ``include/monkeypose.h``)
"""
from . import weights  # noqa: F401
from . import _lib  # noqa: F401
from . import hgru_pose  # noqa: F401
from . import hgru_module  # noqa: F401
from . import train_dense_networks  # noqa: F401
from . import train_hier_networks  # noqa: F401
from . import train_dense_hier_networks  # noqa: F401
from . import train_cnn_networks_hgru  # noqa: F401
from . import monkeydetector  # noqa: F401
from . import pose_evaluation  # noqa: F401
from . import parallel  # noqa: F401
from . import tf_checkpoint  # noqa: F401
from . import data_loader  # noqa: F401

__all__ = ["hgru_pose", "hgru_module", "train_dense_networks", "train_hier_networks", "train_cnn_networks_hgru", "weights", "_lib"]
