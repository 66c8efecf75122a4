from llampc.params.orca import ORCA  # noqa: F401
