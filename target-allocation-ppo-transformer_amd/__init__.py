"""MI355X-native rollout hot path of Dingyf717/target-allocation-ppo-transformer.

Put this directory on sys.path: `uavhip` is the package; `configs`, `envs`, `agents` and `networks`
are drop-in replacements for the reference's modules of the same names, so the reference's
main_train.py runs unchanged."""
