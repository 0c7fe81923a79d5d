from flexflow_train_amd.frontends.keras import *  # noqa: F401,F403
