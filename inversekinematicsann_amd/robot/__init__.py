"""Robot description (robot/robot.py of the reference) and synthetic inputs."""
