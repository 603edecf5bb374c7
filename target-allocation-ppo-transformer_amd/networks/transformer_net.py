"""Drop-in for the reference's networks/transformer_net.py (same class name, state_dict keys and
initialisation; get_action runs the fused HIP forward)."""
from uavhip.policy import TransformerActorCritic, _ortho as init_layer, _Trunk as TransformerBlock  # noqa: F401
