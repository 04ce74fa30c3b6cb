def register_ffmp():
    """gym.envs.registration.register(id='FFMP-v0', entry_point='gym_ffmp.envs:FFMP')."""
    try:
        from gym.envs.registration import register
    except Exception:  # noqa: BLE001 - gym is optional
        return False
    try:
        register(id="FFMP-v0", entry_point="gym_ffmp.envs:FFMP")
    except Exception:  # noqa: BLE001 - already registered
        pass
    return True
