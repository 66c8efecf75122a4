"""ORCA 1:43 vehicle constants (reference: llampc/params/orca.py:8-84)."""


def ORCA(control='pwm'):
    """Parameter dict of the ETH ORCA car; ``control`` 'pwm' (Dynamic) or 'acc'."""
    if control == 'pwm':
        max_inputs, min_inputs = [1., 0.35], [-0.1, -0.35]
    elif control == 'acc':
        max_inputs, min_inputs = [5., 0.35], [-5., -0.35]
    else:
        raise NotImplementedError('choose control as "pwm" for Dynamic model and "acc" for Kinematic model')
    return {
        'lf': 0.029, 'lr': 0.033, 'mass': 0.041, 'Iz': 27.8e-6,
        'Bf': 2.579, 'Br': 3.3852, 'Cf': 1.2, 'Cr': 1.2691, 'Df': 0.192, 'Dr': 0.1737,
        'Cm1': 0.287, 'Cm2': 0.0545, 'Cr0': 0.0518, 'Cr2': 0.00035,
        'max_acc': 5., 'min_acc': -5., 'max_pwm': 1., 'min_pwm': -0.1,
        'max_steer': 0.35, 'min_steer': -0.35, 'max_steer_vel': 5.,
        'max_inputs': max_inputs, 'min_inputs': min_inputs,
        'max_rates': [None, 5.], 'min_rates': [None, -5.],
    }
