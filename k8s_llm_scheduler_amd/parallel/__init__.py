from .comm import CollectiveError, ControlChannel, TPGroup, init_from_env, make_control_channel  # noqa: F401
